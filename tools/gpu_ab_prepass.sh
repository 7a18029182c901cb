mkdir -p gpurun_out/abl2
: > gpurun_out/abl2/res.txt
for rep in 1 2 3 4; do
  for v in "X=1" "CCJ_PREPASS=1"; do
    env $v timeout -k 10 200 python3 tools/level_profile.py 200 > gpurun_out/abl2/out.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/abl2/out.txt; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl2/out.txt').readline()); print('%-28s fill %.2f min %.2f level %.2f' % (sys.argv[1], d['fill_ms_median'], d['fill_ms_min'], d['level4d_ms_uninstrumented']))" "$v" | tee -a gpurun_out/abl2/res.txt
  done
done
