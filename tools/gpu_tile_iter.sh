# one iteration on the k_iltile path: parity (tiles mode), A/B fill timings, SQ counters of k_iltile
mkdir -p gpurun_out
bash tools/gpu_tile_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM"
rm -rf gpurun_out/tpmc
CCJ_ILOOP_TILES=1 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "k_iltile" --pmc $C -d gpurun_out/tpmc -o p -- python3 tools/fold_once.py 200 > gpurun_out/tpmc.log 2>&1 || { echo PMC FAIL; tail -5 gpurun_out/tpmc.log; exit 1; }
f=$(find gpurun_out/tpmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
tot = defaultdict(float); disp=set(); dur={}
for r in csv.DictReader(open(sys.argv[1])):
    tot[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print("k_iltile dispatches", len(disp), "avg_us", sum(dur.values())/max(len(dur),1)/1e3)
print(" ".join("%s=%.4g" % (k.replace("SQ_",""), tot[k] / max(len(disp),1)) for k in sorted(tot)))
PY
