# Full check + write audit: GPU suite, smoke, headline bench, then tools/gpu_write_audit.sh
mkdir -p gpurun_out
echo "== pytest" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== bench" && timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && \
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['breakdown_ms']['fill_device'],d['roofline']['frac'],d['nt_per_s'])" && \
echo "== write audit" && bash tools/gpu_write_audit.sh
