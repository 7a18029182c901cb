# GPU verification chain: bounds-checked fold, GPU parity suite, per-level profile, short bench.
# Every GPU step has its own time limit; any failure ends the chain.
mkdir -p gpurun_out
timeout -k 10 300 python tools/dbg_check.py > gpurun_out/dbg.log 2>&1 && tail -2 gpurun_out/dbg.log && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log && \
timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/levels.txt 2>&1 && cat gpurun_out/levels.txt && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err && cat gpurun_out/bench2.json
rc=$?
[ $rc -ne 0 ] && { tail -5 gpurun_out/pytest_gpu.log 2>/dev/null; tail -5 gpurun_out/bench2.err 2>/dev/null; }
exit $rc
