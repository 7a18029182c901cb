# Iteration loop on the GPU box: a parity subset (matrix hashes vs the reference at small n, the
# BASELINE-size goldens, sharded simulation) and the headline bench.  Extra pytest -k filter: $1
mkdir -p gpurun_out
K=${1:-"parity or large or configs or shard"}
echo "== pytest -k '$K'" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_iter.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_iter.log; [ $rc -eq 0 ]; } && \
echo "== bench" && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err && \
python -c "import json;d=json.load(open('gpurun_out/bench_iter.json'));print('ms/step',d['ms_per_step'],'fill',d['breakdown_ms']['fill_device'],'lvl',d['breakdown_ms']['level4d_levels'],'iloop(instr)',d['breakdown_ms']['iloop_kernels_instrumented_fold'],'mfe',d['mfe'])"
