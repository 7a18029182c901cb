# GPU suite + smoke + headline bench (one JSON line), each step under its own time limit.
mkdir -p gpurun_out
echo "== pytest" && { timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== bench" && timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['breakdown_ms']['fill_device'],d['roofline']['frac'],d['cpu_baseline']['cores'],d['cpu_baseline']['value'],d['nt_per_s'])"
