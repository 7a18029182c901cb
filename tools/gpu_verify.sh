# GPU verification as the driver runs it: pytest -m gpu (all, or the test files given), smoke(),
# then the default bench line (gpurun_out/bench.json).  CONFIGS=1 adds the secondary BASELINE
# configs (tools/gpu_configs.sh).  Each GPU step has its own time limit; the first failure ends it.
#   bash tools/gpu_verify.sh [tests/test_x.py ...]
mkdir -p gpurun_out
T="${*:-tests}"
echo "== pytest $T" && { timeout -k 10 1200 python -u -m pytest $T -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));print('step', d['ms_per_step'], 'fill', d['breakdown_ms']['fill_device'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['cores'], d['cpu_baseline']['value'])" || exit 1
if [ "${CONFIGS:-0}" = 1 ]; then bash tools/gpu_configs.sh || exit 1; fi
