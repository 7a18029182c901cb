#!/bin/bash
# A/B of PF library variants on one box: fill time + per-kernel averages (rocprofv3 kernel trace).
# usage (on the GPU box): tools/pf_ab.sh N variant ...   ("-" = the default libccj_hip.so)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
n=$1; shift
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  d=gpurun_out/pfab/${v:-default}
  mkdir -p $d
  CCJ_LIB_VARIANT=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- \
    python3 tools/pf_time.py $n $n > $d/run.log 2>&1 || exit 1
  echo "== ${v:-default}"; grep "fill" $d/run.log
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-4 "$f" | sed -n 2,6p
done
