# Round profile artifacts (copied into profiles/ by tools/make_profiles.py):
#   kt    : rocprofv3 --kernel-trace --stats of the bench command
#   fetch : --pmc FETCH_SIZE, write: --pmc WRITE_SIZE (separate passes) on k_level4d / k_iltile (k_iloop)
#   bench : the default bench line (with the CPU baseline)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
K="k_level4d|k_iloop|k_iltile|k_pterm|k_ppush|k_diag2d"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- $B > gpurun_out/prof/bench_kt.json 2> gpurun_out/prof/bench_kt.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o f -- $B > gpurun_out/prof/fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc WRITE_SIZE -d gpurun_out/prof/write -o w -- $B > gpurun_out/prof/write.log 2>&1 && \
timeout -k 10 900 python3 bench.py > gpurun_out/prof/bench_full.json 2> gpurun_out/prof/bench_full.err
rc=$?
echo "profile rc=$rc"
cat gpurun_out/prof/bench_full.json
exit $rc
