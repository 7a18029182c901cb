# usage: tools/gpu_abl.sh VARIANT... ("" = default lib); 5-fill medians of tools/level_profile.py 200
mkdir -p gpurun_out
for v in "$@"; do
  [ "$v" = base ] && v=""
  CCJ_LIB_VARIANT=$v timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/abl.txt 2>&1 || { cat gpurun_out/abl.txt; exit 1; }
  echo "== '$v'"; head -1 gpurun_out/abl.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d[k],2) for k in ('fill_ms_median','fill_ms_min','level4d_ms_uninstrumented','fill_ms_instrumented')})"
done
