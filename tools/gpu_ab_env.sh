# Alternating fill medians (tools/level_profile.py 200) of env settings on one box:
#   bash tools/gpu_ab_env.sh "X=1" "CCJ_FOO=1" ...   (3 rounds)
for rep in 1 2 3; do
  for v in "$@"; do
    env $v timeout -k 10 200 python3 tools/level_profile.py 200 > gpurun_out/ab.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab.txt; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.txt').readline()); print('%-24s fill %.2f min %.2f' % (sys.argv[1], d['fill_ms_median'], d['fill_ms_min']))" "$v"
  done
done
