"""Per-wave timeline of one level of the n=200 fill (VERDICT r5 Next 1: measure the level's tail first).

Needs the measurement build (`tools/ablate.sh tl:-DCCJ_WG_TIMELINE` -> ccj_amd/lib/libccj_hip_tl.so, run
with CCJ_LIB_VARIANT=tl): every wave of k_level4d / k_level4d_lead at the armed level stamps the 100 MHz
constant clock (s_memrealtime) at entry and exit; so does every wave of the side kernels around it
(k_iloop(L+1..L+3), k_ppush(L-1..L), k_diag2d(L-1..L)), which gives the whole machine's occupancy over the
level's window ("window": resident waves per kernel family in 20 bins from the plain launch's first start
to the leader launch's last end).

usage: CCJ_LIB_VARIANT=tl python tools/wg_timeline.py [n] [level ...]  -> one JSON line per level
       (or [n] all: every level, one fold each, compact figures: spans, mean resident waves per family):
  span: first wave start -> last wave end of each launch (us)
  ablk_finish: per a-block, when its last wave ended (us from the plain launch's first start), and its scan roles
  busy: the number of waves resident over time in 20 bins per launch (a level's tail shows as a falling count)
  tail: the fraction of the leader launch's span during which fewer than 25% / 50% of its peak waves run
"""
import ctypes
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ccj_amd import W_final, lib  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


class Stamp(ctypes.Structure):
    _fields_ = [("t0", ctypes.c_uint64), ("t1", ctypes.c_uint64), ("meta", ctypes.c_uint64), ("hw", ctypes.c_uint64)]


def waves_of(L, kind, cap):
    buf = (Stamp * cap)()
    if L.ccjk_tl_read(kind, buf, cap) != 0:
        raise RuntimeError("ccjk_tl_read failed")
    return [(s.t0, s.t1, s.meta, s.hw) for s in buf if s.t0]


def busy_curve(ws, t_lo, t_hi, bins=20):
    out = []
    w = (t_hi - t_lo) / bins
    for b in range(bins):
        lo, hi = t_lo + b * w, t_lo + (b + 1) * w
        # wave-time inside the bin / bin width = mean resident waves
        occ = sum(max(0.0, min(t1, hi) - max(t0, lo)) for t0, t1, _, _ in ws) / w
        out.append(round(occ, 1))
    return out


FAMILIES = ["plain", "lead", "iloop+1", "iloop+2", "iloop+3", "ppush-1", "ppush", "diag"]


def window(kinds, lo, hi, bins=20):
    out = {}
    for name, ws in zip(FAMILIES, kinds):
        c = busy_curve(ws, lo, hi, bins) if ws else [0.0] * bins
        if any(c):
            out[name] = c
        if ws:
            out[name + "_span_us"] = [round((min(w[0] for w in ws) - lo) * TICK_US, 1), round((max(w[1] for w in ws) - lo) * TICK_US, 1)]
    return out


def analyse(t, plain, lead):
    base = min(w[0] for w in plain + lead)
    res = {"level": t}
    for name, ws in (("plain", plain), ("lead", lead)):
        if not ws:
            continue
        lo, hi = min(w[0] for w in ws), max(w[1] for w in ws)
        work = [w for w in ws if w[2] != 0xFFFFFFFF and not (w[2] >> 20) & 1]
        durs = sorted((w[1] - w[0]) * TICK_US for w in work)
        res[name] = {
            "start_us": round((lo - base) * TICK_US, 2), "end_us": round((hi - base) * TICK_US, 2),
            "span_us": round((hi - lo) * TICK_US, 2), "waves": len(ws), "working_waves": len(work),
            "wave_us_median": round(durs[len(durs) // 2], 2) if durs else 0,
            "wave_us_p90": round(durs[int(len(durs) * 0.9)], 2) if durs else 0,
            "wave_us_max": round(durs[-1], 2) if durs else 0,
            "cus": len({((w[3] >> 8) & 0xFF, w[3] >> 32) for w in ws}),  # (CU, SH, SE) x XCD
            "busy": busy_curve(ws, lo, hi),
        }
        if name == "lead" and ws:
            curve = busy_curve(ws, lo, hi, bins=100)
            pk = max(curve)
            res[name]["tail_frac_below_25pct"] = sum(1 for c in curve if c < 0.25 * pk) / len(curve)
            res[name]["tail_frac_below_50pct"] = sum(1 for c in curve if c < 0.5 * pk) / len(curve)
    fin = {}
    for ws in (plain, lead):
        for t0, t1, meta, _ in ws:
            if meta == 0xFFFFFFFF or (meta >> 20) & 1:
                continue
            a = meta & 1023
            roles = (meta >> 13) & 3, (meta >> 15) & 3
            e = (t1 - base) * TICK_US
            if a not in fin or e > fin[a][0]:
                fin[a] = (e, roles)
    res["ablk_finish"] = {str(a): [round(fin[a][0], 2), list(fin[a][1])] for a in sorted(fin)}
    f = sorted(v[0] for v in fin.values())
    if f:
        res["ablk_finish_spread_us"] = {"min": round(f[0], 2), "median": round(f[len(f) // 2], 2), "max": round(f[-1], 2)}
    return res


def summary(t, kinds):
    """Compact per-level figures for a whole-fold scan (usage: ... n all): the level's span, its two
    launches' spans, and the machine's mean resident waves per family over the level (wave-us / span)."""
    plain, lead = kinds[0], kinds[1]
    if not plain and not lead:
        return None
    lo = min(w[0] for w in plain + lead)
    hi = max(w[1] for w in plain + lead)
    span = (hi - lo) * TICK_US
    out = {"level": t, "span_us": round(span, 1)}
    for name, ws in zip(FAMILIES, kinds):
        if not ws:
            continue
        wus = sum(max(0, min(w[1], hi) - max(w[0], lo)) for w in ws) * TICK_US
        out[name + "_mean_waves"] = round(wus / span, 1) if span > 0 else 0
    for name, ws in (("plain", plain), ("lead", lead)):
        if ws:
            out[name + "_span_us"] = round((max(w[1] for w in ws) - min(w[0] for w in ws)) * TICK_US, 1)
            work = [w for w in ws if w[2] != 0xFFFFFFFF and not (w[2] >> 20) & 1]
            if work:
                out[name + "_wave_us_max"] = round(max((w[1] - w[0]) * TICK_US for w in work), 1)
                out[name + "_wave_us_mean"] = round(sum((w[1] - w[0]) * TICK_US for w in work) / len(work), 1)
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    scan_all = len(sys.argv) > 2 and sys.argv[2] == "all"
    levels = list(range(n - 2)) if scan_all else ([int(x) for x in sys.argv[2:]] or [60, 100, 140])
    L = lib()
    L.ccjk_tl_arm.argtypes = [ctypes.c_int]
    L.ccjk_tl_read.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    cap = L.ccjk_tl_cap()
    r = random.Random(5)
    seq = "".join(r.choice("ACGU") for _ in range(n))
    wf = W_final(seq, 2, params="Turner04")
    wf.ccj()  # warm-up
    for t in levels:
        if L.ccjk_tl_arm(t) != 0:
            raise RuntimeError("ccjk_tl_arm failed")
        wf.ccj()
        kinds = [waves_of(L, k, cap) for k in range(L.ccjk_tl_kinds())]
        if scan_all:
            sm = summary(t, kinds)
            if sm:
                sm["fill_ms"] = wf.timing()["fill_ms"]
                print(json.dumps(sm), flush=True)
            continue
        res = analyse(t, kinds[0], kinds[1])
        lo = min(w[0] for w in kinds[0] + kinds[1])
        hi = max(w[1] for w in kinds[0] + kinds[1])
        res["window"] = window(kinds, lo, hi)
        res["n"] = n
        res["fill_ms"] = wf.timing()["fill_ms"]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
