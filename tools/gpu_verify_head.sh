# HEAD check: full GPU suite, smoke, one default bench line
mkdir -p gpurun_out
echo "== pytest" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err && cut -c1-300 gpurun_out/bench_head.json
