"""The band-sharded exchange priced on one GPU: every rank of a fold is its own
context in one process (ccj_amd.LocalGroup, one host thread per rank; the real sharded path: own
blocks; per level an edge gather on the level stream and a bulk gather on a side stream, each packed and
unpacked with records and copies).  With timing mode 2 each rank records, per level, the level span,
the edge exchange's part of it and the bulk exchange's time on its own stream (ccj_exchange_times).

The in-process group moves slices with device-to-device copies between two host barriers per level,
on the one GPU all ranks share, so this prices pack + copy + unpack and the per-level
synchronisation, not RCCL over xGMI (unmeasured: 1-GPU boxes only).

usage: python tools/xch_time.py N:G [N:G ...]   (default 200:4 200:8 300:4); one JSON line each
"""
import ctypes
import json
import os
import random
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ccj_amd import LocalGroup, W_final, lib  # noqa: E402


def run(n, G, seed=5):
    r = random.Random(seed)
    seq = "".join(r.choice("ACGU") for _ in range(n))
    L = lib()
    L.ccj_exchange_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                     ctypes.c_int]
    L.ccj_level_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    L.ccj_exchange_layout.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_longlong)]
    g = LocalGroup(G)
    ranks = [W_final(seq, 2, params="Turner04", shard_world=G, shard_rank=q, local_group=g) for q in range(G)]
    out = {}
    try:
        for wf in ranks:
            wf.set_timing(2)
        errs = []

        def worker(w):
            try:
                w.fill()
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        for rep in range(2):  # the first fill warms up; the second is reported
            th = [threading.Thread(target=worker, args=(wf,), daemon=True) for wf in ranks]
            for x in th:
                x.start()
            for x in th:
                x.join(timeout=600)
            if any(x.is_alive() for x in th):
                raise RuntimeError("a rank did not finish its fill within 600 s")
            if errs:
                raise RuntimeError(errs)
        nlev = n - 2
        lev = [(ctypes.c_double * nlev)() for _ in ranks]
        xch = [(ctypes.c_double * nlev)() for _ in ranks]
        xbk = [(ctypes.c_double * nlev)() for _ in ranks]
        for q, wf in enumerate(ranks):
            L.ccj_level_times(wf._h, lev[q], None, nlev)
            L.ccj_exchange_times(wf._h, xch[q], xbk[q], nlev)
        fills = [wf.timing()["fill_ms"] for wf in ranks]
        vol = [0, 0]
        for t in range(nlev):
            for part in (0, 1):
                o = (ctypes.c_longlong * 3)()
                L.ccj_exchange_layout(n, t, G, part, o)
                vol[part] += 2 * o[2] * G  # bytes each rank receives per level and part (the gathered buffer)
        # per level: the slowest rank's exchange share (the exchange ends together on every rank)
        xl = [max(xch[q][t] for q in range(G)) for t in range(nlev)]
        ll = [max(lev[q][t] for q in range(G)) for t in range(nlev)]
        mid = [t for t in range(nlev) if nlev // 3 <= t < 2 * nlev // 3]
        bl = [max(xbk[q][t] for q in range(G)) for t in range(nlev)]
        out = {"n": n, "G": G, "fill_ms_max": max(fills), "fill_ms_min": min(fills),
               "level_span_ms_sum": sum(ll), "exchange_ms_sum": sum(xl),
               "exchange_share": sum(xl) / sum(ll) if sum(ll) else None,
               "exchange_us_per_level_mean": 1e3 * sum(xl) / nlev,
               "exchange_us_per_level_mid_third": 1e3 * sum(xl[t] for t in mid) / max(1, len(mid)),
               "bulk_exchange_us_per_level_mean": 1e3 * sum(bl) / nlev,
               "gathered_GB_per_rank_edge": vol[0] / 1e9, "gathered_GB_per_rank_bulk": vol[1] / 1e9,
               "note": "in-process group on one GPU: slices moved by D2D copies between host barriers, all ranks sharing the GPU; "
                       "exchange_* = the edge part on the level stream (the critical path), bulk_* = the bulk part on its "
                       "side stream (overlaps the next level); RCCL/xGMI unmeasured"}
    finally:
        for wf in ranks:
            wf.close()
        g.close()
    return out


if __name__ == "__main__":
    for arg in sys.argv[1:] or ["200:4", "200:8", "300:4"]:
        n, G = (int(x) for x in arg.split(":"))
        print(json.dumps(run(n, G)), flush=True)
