# Alternating fill timings (tools/level_profile.py, n=200) of k_iltile variants against the default
# work items: each argument is an env assignment list, e.g. "CCJ_ILOOP_TILES=1 CCJ_LIB_VARIANT=tg8"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "CCJ_ILOOP_TILES=0" "$@"; do
    env $v timeout -k 10 200 python3 tools/level_profile.py 200 > gpurun_out/tile_var.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/tile_var.txt; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/tile_var.txt').readline()); print('%-50s fill %.2f min %.2f iloop(instr) %.2f' % (sys.argv[1], d['fill_ms_median'], d['fill_ms_min'], d.get('iloop_ms', -1)))" "$v"
  done
done
