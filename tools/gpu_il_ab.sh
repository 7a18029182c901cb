# k_iloop (default) vs k_iltile (CCJ_ILOOP_TILES=1): parity at the BASELINE sizes, then fill timings
mkdir -p gpurun_out
echo "== pytest large" && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "large or items" > gpurun_out/pytest_il.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_il.log; [ $rc -eq 0 ]; } && \
for v in "X=1" "CCJ_ILOOP_TILES=1" "X=1" "CCJ_ILOOP_TILES=1"; do
  env $v timeout -k 10 200 python3 tools/level_profile.py 200 > gpurun_out/il_ab.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/il_ab.txt; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/il_ab.txt').readline()); print('%-22s fill %.2f min %.2f iloop(instr) %.2f' % (sys.argv[1], d['fill_ms_median'], d['fill_ms_min'], d.get('iloop_ms', -1)))" "$v"
  grep "sum level" gpurun_out/il_ab.txt
done
