#!/bin/bash
# PMC passes (one counter group per run) over the PF fill at n=$1, library variant $2 ("-" = default).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
n=$1; v=$2; [ "$v" = "-" ] && v=""
i=0
for pmc in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1)); d=gpurun_out/pfpmc/p$i; mkdir -p $d
  CCJ_LIB_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $d -o p -- python3 tools/pf_time.py $n > $d/run.log 2>&1 || exit 1
done
