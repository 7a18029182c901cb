# Aggregate throughput of k independent fold processes sharing one GPU (bench.py --gpus k on a
# 1-GPU box: every rank maps to device 0).  Tests whether the n=200 fill leaves the GPU idle.
mkdir -p gpurun_out/probe
for k in 1 2 3 4; do
  timeout -k 10 300 python bench.py --gpus $k --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/probe/g$k.json 2> gpurun_out/probe/g$k.err || exit 1
  python - "$k" <<'PY'
import json, sys
k = sys.argv[1]
d = json.loads(open(f"gpurun_out/probe/g{k}.json").read().strip().splitlines()[-1])
print(k, "ms/step", round(d["ms_per_step"], 2), "seq/s", round(d["sequences_per_s"], 1), "cells/s", round(d["value"] / 1e9, 3))
PY
done
