"""Projection of the band-sharded fill of one long sequence over G GPUs (VERDICT r5 Next 2).

Inputs: the measured 1-GPU span of every level of an n-nt fill on the level stream (tools/level_profile.py
with CCJ_PROFILE_DUMP=...; lev_done[t-1] -> lev_done[t], i.e. the level chain's critical path with its
waits for k_iloop / k_diag2d), and the shipped exchange geometry (ccj_exchange_layout: the edge and bulk
slices of every level).  Model, per level t, for G ranks:
  compute(t) = span_1gpu(t) / G                  (every kernel of the fill partitions its work: a-blocks,
                                                   k_iloop items, k_ppush outer indices, k_diag2d intervals)
  edge(t)    = LAT + slice_edge(t) / BW          (on the level stream: the critical path)
  bulk(t)    = LAT + slice_bulk(t) / BW          (side stream; exposed only beyond the next level's compute)
  fill(G)    = sum_t compute(t) + edge(t) + max(0, bulk(t) - compute(t+1))
An all-gather over a fully connected xGMI node moves every rank's slice to each peer on its own link at
once (G-1 <= 7 links per GPU), so its time is one slice over one link (BW) plus a collective latency (LAT).
Assumptions (no multi-GPU box was available to measure them): BW = 100 GB/s of the ~153 GB/s per xGMI link
(MI355X_MICROARCH.md), LAT = 30 us per RCCL all-gather; both are arguments.  Perfect partitioning is the
optimistic side; each rank's replica of the whole 4-D state (the unpack) is what limits n, not this model.

usage: python tools/shard_projection.py levels_n400.json [BW_GBs LAT_us]  -> one JSON object
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    bw = float(sys.argv[2]) * 1e9 if len(sys.argv) > 2 else 100e9
    lat = float(sys.argv[3]) * 1e-6 if len(sys.argv) > 3 else 30e-6
    d = json.load(open(src))
    n, span = d["n"], [x * 1e-3 for x in d["level_ms"]]
    L = ctypes.CDLL(os.path.join(ROOT, "ccj_amd", "lib", "libccj_hip.so"))
    L.ccj_exchange_layout.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_longlong)]
    t1 = sum(span)
    out = {"n": n, "source": os.path.basename(src), "fill_1gpu_ms": d["fill_ms"], "level_chain_1gpu_ms": t1 * 1e3,
           "assumed_link_GBs": bw / 1e9, "assumed_allgather_latency_us": lat * 1e6, "G": {}}
    for G in (2, 4, 8):
        slices = []
        for t in range(len(span)):
            o = [(ctypes.c_longlong * 3)() for _ in range(2)]
            for part in (0, 1):
                assert L.ccj_exchange_layout(n, t, G, part, o[part]) == 0
            slices.append((2 * o[0][2], 2 * o[1][2]))  # bytes per rank's slice: edge, bulk
        comp = [s / G for s in span]
        edge = [lat + e / bw for e, _ in slices]
        bulk = [lat + b / bw for _, b in slices]
        fill = 0.0
        exposed_bulk = 0.0
        for t in range(len(span)):
            nxt = comp[t + 1] if t + 1 < len(span) else 0.0
            xb = max(0.0, bulk[t] - nxt)
            exposed_bulk += xb
            fill += comp[t] + edge[t] + xb
        one_slice = [lat + (e + b) / bw for e, b in slices]  # round 5: the whole level in one all-gather, serial
        fill_r5 = sum(c + x for c, x in zip(comp, one_slice))
        out["G"][str(G)] = {
            "fill_ms": fill * 1e3, "speedup_vs_1gpu_level_chain": t1 / fill,
            "edge_ms_sum": sum(edge) * 1e3, "bulk_ms_sum": sum(bulk) * 1e3, "bulk_exposed_ms": exposed_bulk * 1e3,
            "edge_bytes_per_rank_per_fold_GB": sum(e for e, _ in slices) * 1e-9,
            "bulk_bytes_per_rank_per_fold_GB": sum(b for _, b in slices) * 1e-9,
            "fill_ms_one_slice_r5": fill_r5 * 1e3, "speedup_one_slice_r5": t1 / fill_r5,
        }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
