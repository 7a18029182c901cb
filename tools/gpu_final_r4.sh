# round-4 final evidence at HEAD: GPU suite + smoke, profiles (tools/gpu_profile.sh), config sweep
mkdir -p gpurun_out
echo "== pytest" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== profile" && bash tools/gpu_profile.sh > gpurun_out/prof_run.txt 2>&1 && tail -1 gpurun_out/prof_run.txt | cut -c1-200 && \
echo "== configs" && bash tools/gpu_configs.sh > gpurun_out/cfg_run.txt 2>&1 && cut -c1-200 gpurun_out/configs.jsonl
