"""Summarise tools/gpu_write_audit.sh: per variant, the median fill (ms) and the HBM bytes per
level of the level chain (k_level4d + k_level4d_lead) and per launch of the side kernels, from the
rocprofv3 FETCH_SIZE / WRITE_SIZE passes (gfx950 factors of tools/make_profiles.py).
usage: python tools/waudit_summary.py [gpurun_out/waudit] [--json profiles/r4_write_audit.json]"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_profiles import FETCH_FACTOR, WRITE_FACTOR, pmc  # noqa: E402


def main(argv):
    d = argv[1] if len(argv) > 1 and not argv[1].startswith("--") else "gpurun_out/waudit"
    out = {}
    for tf in sorted(glob.glob(os.path.join(d, "time_*.txt"))):
        v = os.path.basename(tf)[5:-4]
        with open(tf) as f:
            tm = json.loads(f.readline())
        rec = {"fill_ms_median": tm["fill_ms_median"], "kernels": {}}
        for c, fac in (("WRITE_SIZE", WRITE_FACTOR), ("FETCH_SIZE", FETCH_FACTOR)):
            fs = glob.glob(os.path.join(d, f"{v}_{c}", "**", "*counter_collection.csv"), recursive=True)
            if not fs:
                continue
            for k, (b, nl) in pmc(fs[0], c).items():
                rec["kernels"].setdefault(k, {})[c.split("_")[0].lower() + "_MB_per_launch"] = fac * b / max(nl, 1) / 1e6
        out[v] = rec
    for v, r in out.items():
        lv = r["kernels"].get("k_level4d_level", {})
        print(f"{v:8s} fill {r['fill_ms_median']:6.2f} ms  level write {lv.get('write_MB_per_launch', 0):6.1f} MB  "
              f"fetch {lv.get('fetch_MB_per_launch', 0):6.1f} MB  | " +
              "  ".join(f"{k} w{x.get('write_MB_per_launch', 0):.1f}/f{x.get('fetch_MB_per_launch', 0):.1f}"
                        for k, x in sorted(r["kernels"].items()) if k not in ("k_level4d_level",)))
    if "--json" in argv:
        with open(argv[argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv)
