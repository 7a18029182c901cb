"""Where the level chain loses time: per-level timeline of the last fold in a rocprofv3 kernel trace.

usage: python tools/trace_timeline.py gpurun_out/tl/<...>_kernel_trace.csv [fold index, default -1]

For each level t of the last fold: the level's kernels (k_level4d, then k_level4d_lead on the
sharing levels), the gap since level t-1 ended, the gap between the level's two launches, and how
late its cross-stream inputs finished relative to the end of level t-1 (k_iloop(t) on st_il,
k_diag2d(t-1) on st_d).  Kernels are matched to levels by dispatch order: the host enqueues
k_diag2d(s), k_iloop(s), k_level4d(s), k_level4d_lead(s), k_pterm(s+3) for every s.
"""
import csv
import re
import statistics as stx
import sys


def kname(full):
    return re.sub(r"^void ", "", full.split("(")[0]).strip()


def main(path, which=-1):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), kname(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    starts = [i for i, (d, k, s, e) in enumerate(rows) if k == "k_init2d"]
    starts.append(len(rows))
    x0 = starts[which - 1] if which < 0 else starts[which]
    x1 = starts[which] if which < 0 else starts[which + 1]
    fold = rows[x0:x1]
    lv = []  # [plain, lead or None, iloop or None, diag or None]
    for x, (d, k, s, e) in enumerate(fold):
        if k != "k_level4d":
            continue
        lead = fold[x + 1] if x + 1 < len(fold) and fold[x + 1][1] == "k_level4d_lead" else None
        il = None  # k_iloop(t): just before level t, or before k_diag2d(t-1) when the diag is joined to st_il
        for y in range(x - 1, max(x - 4, -1), -1):
            if fold[y][1] == "k_iloop":
                il = fold[y]
                break
            if fold[y][1].startswith("k_level4d"):
                break
        dg = None
        for y in range(x - 1, max(x - 4, -1), -1):
            if fold[y][1] == "k_diag2d":
                dg = fold[y]
                break
        lv.append(((s, e), (lead[2], lead[3]) if lead else None, (il[2], il[3]) if il else None, (dg[2], dg[3]) if dg else None))
    t0 = fold[0][2]
    gaps, inner, spans, il_late, dg_late, crit = [], [], [], [], [], {"prev_level": 0, "iloop": 0, "diag2d": 0}
    prev_end = None
    prev_dg = None
    out = []
    for t, (pl, ld, il, dg) in enumerate(lv):
        start = pl[0] if ld is None else min(pl[0], ld[0])
        end = pl[1] if ld is None else max(pl[1], ld[1])
        spans.append(end - start)
        if ld is not None:
            inner.append(ld[0] - pl[1])
        if prev_end is not None:
            g = start - prev_end
            gaps.append(g)
            li = (il[1] - prev_end) if il else None
            ldg = (prev_dg[1] - prev_end) if prev_dg else None
            if li is not None:
                il_late.append(li)
            if ldg is not None:
                dg_late.append(ldg)
            who = max([("prev_level", 0), ("iloop", li if li is not None else -1e18), ("diag2d", ldg if ldg is not None else -1e18)],
                      key=lambda z: z[1])[0]
            crit[who] += 1
            out.append((t, (start - t0) / 1e3, (end - start) / 1e3, g / 1e3, (li or 0) / 1e3, (ldg or 0) / 1e3,
                        ((ld[0] - pl[1]) / 1e3) if ld else None))
        prev_end = end
        prev_dg = dg
    fold_ms = (max(e for d, k, s, e in fold) - t0) / 1e6
    print(f"fold {fold_ms:.2f} ms over {len(lv)} levels; level spans sum {sum(spans)/1e6:.2f} ms; "
          f"gaps sum {sum(gaps)/1e6:.2f} ms (median {stx.median(gaps)/1e3:.1f} us)")
    if inner:
        print(f"plain->lead gap: median {stx.median(inner)/1e3:.1f} us, sum {sum(inner)/1e6:.2f} ms over {len(inner)} levels")
    print(f"k_iloop(t) end - level(t-1) end: median {stx.median(il_late)/1e3:.1f} us, "
          f"late (>0) on {sum(1 for v in il_late if v > 0)} levels, sum of lateness {sum(v for v in il_late if v > 0)/1e6:.2f} ms")
    print(f"k_diag2d(t-1) end - level(t-1) end: median {stx.median(dg_late)/1e3:.1f} us, "
          f"late on {sum(1 for v in dg_late if v > 0)} levels, sum {sum(v for v in dg_late if v > 0)/1e6:.2f} ms")
    print("critical input per level:", crit)
    print("   t   start_us  span_us   gap_us  il_late  dg_late  inner_gap")
    for r in out[:: max(1, len(out) // 40)]:
        print("%4d %10.1f %8.1f %8.1f %8.1f %8.1f %s" % (r[0], r[1], r[2], r[3], r[4], r[5], "" if r[6] is None else "%8.1f" % r[6]))


if __name__ == "__main__":
    # which fold: -1 = last (tools/level_profile.py's last fold is the marker-instrumented one), -2 ...
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -1)
