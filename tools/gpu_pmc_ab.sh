# Per-kernel HBM traffic A/B: tools/gpu_pmc_ab.sh KERNEL_REGEX "VAR=a" "VAR=b" ...
# For each variant: FETCH_SIZE and WRITE_SIZE passes (separate runs) over tools/level_profile.py
# (CCJ_PROFILE_REPS=1 -> 3 folds traced), then tools/pmc_summary.py per kernel name.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K="$1"; shift
mkdir -p gpurun_out/pab
for v in "$@"; do
  tag=$(echo "$v" | tr -c 'A-Za-z0-9' '_')
  for c in FETCH_SIZE WRITE_SIZE; do
    env $v CCJ_PROFILE_REPS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc $c \
      -d gpurun_out/pab/$tag/$c -o p -- python3 tools/level_profile.py 200 > gpurun_out/pab/$tag.$c.log 2>&1 || { echo "FAIL $v $c"; tail -5 gpurun_out/pab/$tag.$c.log; exit 1; }
  done
  for kn in $(echo "$K" | tr '|' ' '); do
    echo "== $v $kn"
    python3 tools/pmc_summary.py 3 $(find gpurun_out/pab/$tag -name '*counter_collection.csv') $kn
  done
done
