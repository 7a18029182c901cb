# PF fill counter passes: FETCH_SIZE and WRITE_SIZE per launch of the four PF kernels over the
# bench.py --pf command (-> tools/make_profiles.py r4 --pf --traffic-only --prof gpurun_out/profpf)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/profpf
B="python3 bench.py --pf --steps 2 --warmup 1 --no-cpu-baseline"
K="k_pf_level|k_pf_iloop|k_pf_pterm|k_pf_diag"
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc FETCH_SIZE -d gpurun_out/profpf/fetch -o f -- $B > gpurun_out/profpf/fetch.log 2>&1 && \
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc WRITE_SIZE -d gpurun_out/profpf/write -o w -- $B > gpurun_out/profpf/write.log 2>&1 && \
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profpf/kt -o kt --output-format csv -- $B > gpurun_out/profpf/kt.log 2>&1 && \
echo "pf counter passes ok"
