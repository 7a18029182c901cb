# Run a subset of the GPU tests (args: test files) plus a short default bench line.
mkdir -p gpurun_out
echo "== pytest $*" && { timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_new.log | tail -40; [ $rc -le 1 ] && [ $rc -eq 0 ]; } && \
echo "== bench" && timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err; rc=$?; cut -c1-900 gpurun_out/bench_new.json; tail -3 gpurun_out/bench_new.err; exit $rc
