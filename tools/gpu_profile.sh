# Round profile artifacts (copied into profiles/ by tools/make_profiles.py):
#   bash tools/gpu_profile.sh [mfe|n400|pf]
#   mfe  (default): kt = --kernel-trace --stats of the bench command, FETCH_SIZE and WRITE_SIZE passes
#                   (separate runs) of the fill kernels, then the default bench line (CPU baseline on)
#   n400          : the two counter passes over bench.py --n 400 --seed 6 (config 5 per GPU)
#   pf            : the counter passes and a kernel trace over bench.py --pf
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
what="${1:-mfe}"
case "$what" in
  mfe)  D=gpurun_out/prof;    B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline";                 K="k_level4d|k_iloop|k_ppush|k_diag2d" ;;
  n400) D=gpurun_out/prof400; B="python3 bench.py --n 400 --seed 6 --steps 1 --warmup 1 --no-cpu-baseline"; K="k_level4d|k_iloop|k_ppush|k_diag2d" ;;
  pf)   D=gpurun_out/profpf;  B="python3 bench.py --pf --steps 2 --warmup 1 --no-cpu-baseline";            K="k_pf_level|k_pf_iloop|k_pf_pterm|k_pf_ppush|k_pf_diag" ;;
  *) echo "usage: gpu_profile.sh [mfe|n400|pf]"; exit 2 ;;
esac
mkdir -p $D
if [ "$what" != n400 ]; then
  timeout -k 10 -s KILL 600 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- $B > $D/bench_kt.json 2> $D/bench_kt.err || { echo "kernel trace failed"; exit 1; }
fi
timeout -k 10 -s KILL 600 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc FETCH_SIZE -d $D/fetch -o f -- $B > $D/fetch.log 2>&1 && \
timeout -k 10 -s KILL 600 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc WRITE_SIZE -d $D/write -o w -- $B > $D/write.log 2>&1 || { echo "counter passes failed"; exit 1; }
if [ "$what" = mfe ]; then
  timeout -k 10 900 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { echo "bench failed"; exit 1; }
  cat $D/bench_full.json
fi
echo "profile $what ok"
