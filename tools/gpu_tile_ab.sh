# k_iltile (CCJ_ILOOP_TILES=1) vs the default k_iloop work items: parity of the tile path on the
# reference goldens (n=100/150, unsharded and band-sharded), then alternating fill timings at n=200.
mkdir -p gpurun_out
echo "== tiles parity" && { timeout -k 10 400 python -u -m pytest tests/test_gpu_items.py -x -q --timeout 380 --timeout-method thread -k tiles > gpurun_out/tile_parity.log 2>&1; rc=$?; tail -3 gpurun_out/tile_parity.log; [ $rc -eq 0 ]; } && \
for v in "CCJ_ILOOP_TILES=0" "CCJ_ILOOP_TILES=1" "CCJ_ILOOP_TILES=0" "CCJ_ILOOP_TILES=1"; do
  env $v timeout -k 10 200 python3 tools/level_profile.py 200 > gpurun_out/tile_ab.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/tile_ab.txt; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/tile_ab.txt').readline()); print('%-22s fill %.2f min %.2f iloop(instr) %.2f' % (sys.argv[1], d['fill_ms_median'], d['fill_ms_min'], d.get('iloop_ms', -1)))" "$v"
done
