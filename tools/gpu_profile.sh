# rocprofv3 runs for profiles/: kernel trace + stats of the bench, then separate PMC passes
# (one counter group per pass, never combined with runtime/sys tracing).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
P="--kernel-trace --output-format csv --kernel-include-regex k_level4d"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_kt.json 2> gpurun_out/prof/bench_kt.err && \
timeout -k 10 600 rocprofv3 $P --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o f -- python3 tools/level_profile.py 200 > gpurun_out/prof/fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 $P --pmc WRITE_SIZE -d gpurun_out/prof/write -o w -- python3 tools/level_profile.py 200 > gpurun_out/prof/write.log 2>&1 && \
timeout -k 10 600 rocprofv3 $P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof/tcc -o tcc -- python3 tools/level_profile.py 200 > gpurun_out/prof/tcc.log 2>&1 && \
timeout -k 10 600 rocprofv3 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/prof/sq -o sq -- python3 tools/level_profile.py 200 > gpurun_out/prof/sq.log 2>&1
rc=$?
echo "profile rc=$rc"
exit $rc
