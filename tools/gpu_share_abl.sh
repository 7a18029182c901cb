mkdir -p gpurun_out
for cfg in "2 ''" "2 r3" "2 r2" "1 r3" "3 r3" "2 r3"; do
  set -- $cfg; ls=$1; v=$(eval echo $2)
  CCJ_LEAD_SPLIT=$ls CCJ_LIB_VARIANT=$v timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/abl.txt 2>&1 || { cat gpurun_out/abl.txt; exit 1; }
  echo "== R-variant '$v' lsplit $ls"; head -1 gpurun_out/abl.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d[k],2) for k in ('fill_ms_median','fill_ms_min','level4d_ms','iloop_ms')})"
done
CCJ_SHARE_SPLITS=-1 timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/abl.txt 2>&1 && echo "== noshare" && head -1 gpurun_out/abl.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d[k],2) for k in ('fill_ms_median','fill_ms_min','level4d_ms','iloop_ms')})"
