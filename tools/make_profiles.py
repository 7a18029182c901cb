"""Copy the round's profile evidence from gpurun_out/prof (tools/gpu_profile.sh) into profiles/.

usage: python tools/make_profiles.py ROUND [--n N --seed S --params P] [--traffic-only] [--prof DIR]
Writes profiles/<ROUND>_kernel_stats.csv (rocprofv3 --stats), profiles/<ROUND>_bench.json (the
bench line), and profiles/traffic.json: FETCH_SIZE/WRITE_SIZE per launch of each profiled kernel,
converted to bytes with the gfx950 calibration of tools/microbench/fetch_calib.hip (FETCH_SIZE
counts half the bytes of coalesced 2/4/16-byte loads; WRITE_SIZE counts 2-byte stores exactly).
bench.py reports profiles/traffic.json's k_level4d figure as roofline.traffic.
"""
import csv
import json
import os
import re
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
            k = kname(r["Kernel_Name"])
            tot[k] += float(r["Counter_Value"]) * 1024.0  # KB -> bytes
            launches[k].add(r["Dispatch_Id"])
            if k == "k_level4d_lead":
                # one level = k_level4d + (on sharing levels) k_level4d_lead: bytes summed under
                # "k_level4d_level", launches counted once per level
                tot["k_level4d_level"] += float(r["Counter_Value"]) * 1024.0
            elif k == "k_level4d":
                tot["k_level4d_level"] += float(r["Counter_Value"]) * 1024.0
                launches["k_level4d_level"].add(r["Dispatch_Id"])
    return {k: (tot[k], len(launches[k])) for k in tot}


def kname(full):
    """'void k_level4d(ccj::DevTables, ...)' -> 'k_level4d'; template arguments dropped ('k_ppush<8, 4>' -> 'k_ppush')"""
    return re.sub(r"^void ", "", full.split("(")[0].split("<")[0]).strip()


def level_spans(trace_csv):
    """Per-level span of the level kernels from the kernel trace: each k_level4d_lead dispatch
    runs beside the k_level4d dispatch of the same level (they overlap in time); the level's
    span is first start to last end, the figure bench.py measures with HIP events on the level
    stream (roofline.avg_launch_us)."""
    plain, lead = [], []
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            k = kname(r["Kernel_Name"])
            iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            if k == "k_level4d":
                plain.append(iv)
            elif k == "k_level4d_lead":
                lead.append(iv)
    plain.sort()
    lead.sort()
    # both launches of a level wait for the same events, so a leader dispatch belongs to the plain
    # dispatch whose start is nearest to its own
    import bisect
    starts = [p[0] for p in plain]
    span = [list(p) for p in plain]
    for s0, e0 in lead:
        x = bisect.bisect_left(starts, s0)
        cand = [y for y in (x - 1, x) if 0 <= y < len(plain)]
        y = min(cand, key=lambda y: abs(starts[y] - s0))
        span[y][0], span[y][1] = min(span[y][0], s0), max(span[y][1], e0)
    spans = [e - s for s, e in span]
    return {"levels": len(spans), "avg_level_span_us": sum(spans) / max(len(spans), 1) / 1e3,
            "plain_dispatches": len(plain), "leader_dispatches": len(lead)}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--prof", default=PROF, help="gpurun_out/prof-style directory (kt/, fetch/, write/)")
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--params", default="Turner04")
    ap.add_argument("--traffic-only", action="store_true", help="only the PMC summary (no stats/bench/spans)")
    ap.add_argument("--pf", action="store_true", help="the partition-function fill (bench.py --pf)")
    a = ap.parse_args()
    rnd, prof = a.round, a.prof
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    headline = (a.n, a.seed, a.params) == (200, 5, "Turner04")
    if not a.traffic_only:
        shutil.copy(os.path.join(prof, "kt", "kt_kernel_stats.csv"), os.path.join(out, f"{rnd}_kernel_stats.csv"))
        with open(os.path.join(prof, "bench_full.json")) as f:
            line = f.read().strip().splitlines()[-1]
        with open(os.path.join(out, f"{rnd}_bench.json"), "w") as f:
            f.write(line + "\n")
    fe = pmc(os.path.join(prof, "fetch", "f_counter_collection.csv"), "FETCH_SIZE")
    wr = pmc(os.path.join(prof, "write", "w_counter_collection.csv"), "WRITE_SIZE")
    cmd = "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline" + (" --pf" if a.pf else "")
    if not headline:
        cmd += f" --n {a.n} --seed {a.seed} --params {a.params}"
    traffic = {"round": rnd, "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- " + cmd,
               "config": {"n": a.n, "seed": a.seed, "params": a.params}, "pf": a.pf,
               "fetch_factor": FETCH_FACTOR, "write_factor": WRITE_FACTOR, "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        fb, fl = fe.get(k, (0.0, 1))
        wb, wl = wr.get(k, (0.0, 1))
        traffic["kernels"][k] = {"launches": fl, "read_bytes_per_launch": FETCH_FACTOR * fb / max(fl, 1),
                                 "write_bytes_per_launch": WRITE_FACTOR * wb / max(wl, 1),
                                 "hbm_bytes_per_launch": FETCH_FACTOR * fb / max(fl, 1) + WRITE_FACTOR * wb / max(wl, 1)}
    name = ("traffic.json" if headline else f"traffic_n{a.n}_s{a.seed}_{a.params}.json") if not a.pf else \
        f"traffic_pf_n{a.n}_s{a.seed}_{a.params}.json"
    with open(os.path.join(out, name), "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))
    if not a.traffic_only:
        sp = level_spans(os.path.join(prof, "kt", "kt_kernel_trace.csv"))
        with open(os.path.join(out, f"{rnd}_level_span.json"), "w") as f:
            json.dump(sp, f, indent=1)
        print(json.dumps(sp, indent=1))


if __name__ == "__main__":
    main()
