# FETCH_SIZE / WRITE_SIZE per known byte count (tools/microbench/fetch_calib.hip)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/calib
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d gpurun_out/calib/f -o f -- ./tools/microbench/fetch_calib > gpurun_out/calib/f.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d gpurun_out/calib/w -o w -- ./tools/microbench/fetch_calib > gpurun_out/calib/w.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/calib/*/*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        kb = float(r["Counter_Value"])
        if r["Kernel_Name"].startswith("k_window"):
            print(f'{r["Kernel_Name"][:40]:40s} {r["Counter_Name"]:11s} {kb*1024/262144:.1f} bytes per wave')
        else:
            print(f'{r["Kernel_Name"][:40]:40s} {r["Counter_Name"]:11s} {kb*1024/2**30:.3f} x 1GiB')
PY
exit $rc
