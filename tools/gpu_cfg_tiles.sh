# BASELINE config sweep (tools/gpu_configs.sh, tile default) plus n=400 with the work items
bash tools/gpu_configs.sh > gpurun_out/cfg_run.txt 2>&1 || { tail -5 gpurun_out/cfg_run.txt; exit 1; }
CCJ_ILOOP_TILES=0 timeout -k 10 600 python bench.py --n 400 --seed 6 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg400_items.json 2>> gpurun_out/cfg.err || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/configs.jsonl"):
    d = json.loads(l)
    print(d["config"]["n"], d["config"]["params"], round(d["ms_per_step"], 2), round(d["breakdown_ms"]["fill_device"], 2), d["mfe"])
d = json.load(open("gpurun_out/cfg400_items.json"))
print("items n400", round(d["ms_per_step"], 2), round(d["breakdown_ms"]["fill_device"], 2), d["mfe"])
PY
