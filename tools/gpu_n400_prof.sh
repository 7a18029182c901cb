# Config 5 (n=400, seed 6) counter passes: FETCH_SIZE and WRITE_SIZE per launch of the fill kernels
# (-> tools/make_profiles.py r4 --n 400 --seed 6 --traffic-only --prof gpurun_out/prof400)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof400
B="python3 bench.py --n 400 --seed 6 --steps 1 --warmup 1 --no-cpu-baseline"
K="k_level4d|k_iloop|k_ppush|k_diag2d"
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc FETCH_SIZE -d gpurun_out/prof400/fetch -o f -- $B > gpurun_out/prof400/fetch.log 2>&1 && \
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc WRITE_SIZE -d gpurun_out/prof400/write -o w -- $B > gpurun_out/prof400/write.log 2>&1 && \
echo "counter passes ok" && tail -1 gpurun_out/prof400/fetch.log | cut -c1-200
