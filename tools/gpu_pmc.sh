# rocprofv3 counter passes (one run per counter set: rocprofv3 does not split sets over passes)
# for the kernels matching a regex, over CMD (default: one n=200 fold), summed per fold by
# tools/pmc_summary.py for each kernel name in KERNELS (default: the regex itself).
#   bash tools/gpu_pmc.sh "k_level4d" "SQ_WAVES SQ_INSTS_VALU" "TCC_HIT_sum TCC_MISS_sum" ...
#   CMD="python3 bench.py --pf --steps 1 --warmup 1 --no-cpu-baseline" FOLDS=2 bash tools/gpu_pmc.sh ...
# Limits per set (gfx950): 8 SQ_, 4 TCC_ (FETCH_SIZE takes 3, WRITE_SIZE 2), 4 TCP_, 2 TA_, 2 TD_.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K="$1"; shift
CMD="${CMD:-python3 tools/fold_once.py 200 1}"
D=gpurun_out/pmc
rm -rf $D && mkdir -p $D
x=0
for set in "$@"; do
  x=$((x + 1))
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc $set -d $D/p$x -o p -- $CMD > $D/p$x.log 2>&1 || { echo "pmc pass $x ($set) failed"; tail -5 $D/p$x.log; exit 1; }
done
for k in ${KERNELS:-$K}; do
  echo "== $k"
  python3 tools/pmc_summary.py "${FOLDS:-1}" $(find $D -name '*counter_collection.csv') "$k"
done
