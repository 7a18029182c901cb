# GPU suite, smoke, headline bench, and fill medians (tools/level_profile.py, 3 runs)
mkdir -p gpurun_out
echo "== pytest" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } && \
echo "== smoke" && timeout -k 10 120 python __graft_entry__.py smoke && \
echo "== bench" && timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && \
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['breakdown_ms']['fill_device'],d['roofline']['frac'],d['nt_per_s'])" && \
for r in 1 2 3; do timeout -k 10 200 python3 tools/level_profile.py 200 > gpurun_out/lp.txt 2>&1 && python3 -c "import json; d=json.loads(open('gpurun_out/lp.txt').readline()); print('fill median %.2f min %.2f' % (d['fill_ms_median'], d['fill_ms_min']))" || exit 1; done
