mkdir -p gpurun_out
echo "== dbg" && timeout -k 10 300 python tools/dbg_check.py > gpurun_out/dbg.log 2>&1 && tail -3 gpurun_out/dbg.log && \
echo "== pytest" && { timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -le 1 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== bench" && timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
