# Level-chain write audit: fill time and rocprofv3 WRITE_SIZE / FETCH_SIZE per
# level for the default library and timing-only builds that drop one buffer's stores
# (tools/ablate.sh: NOREC = loop records, NOACC = split-sharing partials, NOCOPY = interior-loop
# copies, NOMAT5 = the 5 matrices no fill kernel reads back).  Results: gpurun_out/waudit/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/waudit
K="k_level4d|k_iltile|k_iloop|k_ppush"
for v in - norec noacc nocopy nomat5; do
  [ "$v" = "-" ] && lv="" || lv=$v
  echo "== ${v}"
  CCJ_LIB_VARIANT=$lv timeout -k 10 120 python3 tools/level_profile.py 200 > gpurun_out/waudit/time_$v.txt 2>&1 || exit 1
  head -1 gpurun_out/waudit/time_$v.txt | cut -c1-300
  for c in WRITE_SIZE FETCH_SIZE; do
    CCJ_LIB_VARIANT=$lv CCJ_PROFILE_REPS=1 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$K" --pmc $c -d gpurun_out/waudit/${v}_$c -o p -- python3 tools/level_profile.py 200 > gpurun_out/waudit/${v}_$c.log 2>&1 || exit 1
  done
done
python3 tools/waudit_summary.py gpurun_out/waudit
