"""Copy the round's profile evidence from gpurun_out/prof (tools/gpu_profile.sh) into profiles/.

usage: python tools/make_profiles.py ROUND      (e.g. r1)
Writes profiles/<ROUND>_kernel_stats.csv (rocprofv3 --stats), profiles/<ROUND>_bench.json (the
bench line), and profiles/traffic.json: FETCH_SIZE/WRITE_SIZE per launch of each profiled kernel,
converted to bytes with the gfx950 calibration of tools/microbench/fetch_calib.hip (FETCH_SIZE
counts half the bytes of coalesced 2/4/16-byte loads; WRITE_SIZE counts 2-byte stores exactly).
bench.py reports profiles/traffic.json's k_level4d figure as roofline.traffic.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")
FETCH_FACTOR = 2.0  # bytes per FETCH_SIZE byte (calibrated)
WRITE_FACTOR = 1.0


def pmc(path, counter):
    tot, launches = defaultdict(float), defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0]
            tot[k] += float(r["Counter_Value"]) * 1024.0  # KB -> bytes
            launches[k].add(r["Dispatch_Id"])
    return {k: (tot[k], len(launches[k])) for k in tot}


def main():
    rnd = sys.argv[1]
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(PROF, "kt", "kt_kernel_stats.csv"), os.path.join(out, f"{rnd}_kernel_stats.csv"))
    with open(os.path.join(PROF, "bench_full.json")) as f:
        line = f.read().strip().splitlines()[-1]
    with open(os.path.join(out, f"{rnd}_bench.json"), "w") as f:
        f.write(line + "\n")
    fe = pmc(os.path.join(PROF, "fetch", "f_counter_collection.csv"), "FETCH_SIZE")
    wr = pmc(os.path.join(PROF, "write", "w_counter_collection.csv"), "WRITE_SIZE")
    traffic = {"round": rnd, "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- "
               "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline",
               "fetch_factor": FETCH_FACTOR, "write_factor": WRITE_FACTOR, "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        fb, fl = fe.get(k, (0.0, 1))
        wb, wl = wr.get(k, (0.0, 1))
        traffic["kernels"][k] = {"launches": fl, "read_bytes_per_launch": FETCH_FACTOR * fb / max(fl, 1),
                                 "write_bytes_per_launch": WRITE_FACTOR * wb / max(wl, 1),
                                 "hbm_bytes_per_launch": FETCH_FACTOR * fb / max(fl, 1) + WRITE_FACTOR * wb / max(wl, 1)}
    with open(os.path.join(out, "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
