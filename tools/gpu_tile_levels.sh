# per-level durations (rocprofv3 kernel trace, one fold at n=200) of k_iloop (items) and k_iltile
# (CCJ_ILOOP_TILES=1), in the concurrent fill, plus their per-fill setup kernels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/tlev; mkdir -p gpurun_out/tlev
for v in items tile; do
  [ $v = tile ] && export CCJ_ILOOP_TILES=1; [ $v = items ] && export CCJ_ILOOP_TILES=0
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlev/$v -o p -- python3 tools/fold_once.py 200 > gpurun_out/tlev/$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/tlev/$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
def load(v):
    f = glob.glob(f"gpurun_out/tlev/{v}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    return rows
def durs(rows, name):
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
A, B = load("items"), load("tile")
a, b = durs(A, "k_iloop"), durs(B, "k_iltile")
for nm in ("k_build_il", "k_items", "k_ie_tiles", "k_precompute_ie"):
    print(nm, "items", round(sum(durs(A, nm)), 1), "tile", round(sum(durs(B, nm)), 1))
print("per 8 levels (us): first level, items, tiles")
for i in range(0, min(len(a), len(b)), 8):
    print(i, round(sum(a[i:i+8]), 1), round(sum(b[i:i+8]), 1))
print("total", round(sum(a), 1), round(sum(b), 1))
PY
