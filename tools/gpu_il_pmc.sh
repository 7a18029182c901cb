# SQ counters of the interior-loop kernels (k_iloop default, k_iltile with CCJ_ILOOP_TILES=1):
# instruction mix and where the waves wait.  One PMC pass per kernel variant.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ilpmc
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM"
for v in tile items; do
  [ $v = tile ] && export CCJ_ILOOP_TILES=1; [ $v = items ] && export CCJ_ILOOP_TILES=0
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "k_iltile|k_iloop" --pmc $C -d gpurun_out/ilpmc/$v -o p -- python3 tools/fold_once.py 200 > gpurun_out/ilpmc/$v.log 2>&1 || exit 1
  f=$(find gpurun_out/ilpmc/$v -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
tot = defaultdict(float); disp=set(); dur={}
for r in csv.DictReader(open(sys.argv[1])):
    tot[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print("dispatches", len(disp), "avg_us", sum(dur.values())/max(len(dur),1)/1e3)
for k in sorted(tot): print(k, "%.4g" % (tot[k] / max(len(disp),1)))
PY
done
