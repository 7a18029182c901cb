# The whole GPU test suite as the driver runs it, smoke, then the secondary configs.
mkdir -p gpurun_out
echo "== pytest" && { timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== configs" && bash tools/gpu_configs.sh
