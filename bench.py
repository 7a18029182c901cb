#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X CCJ engine (BASELINE.json metric/config 3).

One "step" = one complete CCJ MFE fold of the 200-nt synthetic RNA (random.Random(5), ACGU) with
rna_Turner04 tables and dangles 2: GPU fill of all 22 four-dimensional gap matrices and the
2-D matrices, exterior W, traceback and bracket emission (on the GPU; the structure string and
MFE are copied back) — everything W_final::ccj() does in the reference.  Inputs are resident in
HBM before the timed region (the context is created during setup).  Every ccj() call returns
only after all of its streams are synchronized, so the barrier + wall clock around the K steps
brackets finished GPU work (the engine's own stream sync plays the role of a device sync).

    python bench.py [--gpus N] [--steps K] [--warmup W]

With N > 1 (torch.distributed.run, one process per GPU) every rank folds its own copy of the
sequence (batch mode, weak scaling, no data-path collective); the barrier and max-over-ranks
timing use torch.distributed (gloo).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import random
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sec/sequence + DP-cells/s at n=200 (Turner04), 1/2/4/8 GPU vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec


def rseq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


def max_over_ranks(elapsed, dist):
    """The job's time: the slowest rank's wall clock over the timed steps (gloo all-reduce MAX)."""
    if dist is None:
        return elapsed
    import torch
    tt = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def job_value(cells, steps, elapsed, world, shard):
    """Whole-job DP-cells/s: batch mode folds one sequence per rank per step, band sharding one
    sequence per step over all ranks."""
    seqs_per_step = 1 if shard else world
    return seqs_per_step * steps * cells / elapsed


def cpu_baseline(n_sample=100, seed=3, params="Turner04"):
    """Reference CPU CCJ (oracle/_ref/ref_driver, compiled from the reference sources) on a bounded
    sample of the same workload; falls back to our C restatement (oracle/ccj_oracle.c)."""
    from ccj_amd import num_cells
    seq = rseq(seed, n_sample)
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    blob = os.path.join(ROOT, "ccj_amd", "params", params + ".ccjp")
    cells = num_cells(n_sample)
    if os.path.exists(drv):
        r = subprocess.run([drv, "fold", "--blob", blob, "--time", seq], capture_output=True, text=True, timeout=900)
        if r.returncode == 0 and "TIME" in r.stderr:
            t = float(r.stderr.split("TIME")[1].split()[0])
            return {"value": cells / t, "unit": "DP-cells/s", "cores": 1, "kind": "reference",
                    "seconds": t, "sample": f"one full reference fold (W_final::ccj) of a {n_sample}-nt random RNA "
                    f"(seed {seed}, {params}, {cells} cells) on 1 host core; the reference is single-threaded"}
    from tests.oracle_lib import OracleFold
    with open(blob, "rb") as f:
        b = f.read()
    t0 = time.perf_counter()
    o = OracleFold(seq, b, 2, 0)
    t = time.perf_counter() - t0
    o.close()
    return {"value": cells / t, "unit": "DP-cells/s", "cores": 1, "kind": "port", "seconds": t,
            "sample": f"C restatement fill of a {n_sample}-nt random RNA (seed {seed}, {params}) on 1 host core"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--params", default="Turner04")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-n", type=int, default=110)
    ap.add_argument("--shard", action="store_true",
                    help="band-shard ONE sequence over all ranks (RCCL all-gather per level, strong scaling) "
                         "instead of one sequence per GPU")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    from ccj_amd import W_final, num_cells, lib, comm_unique_id
    import ctypes

    seq = rseq(a.seed, a.n)
    shard = a.shard and world > 1
    if shard:
        obj = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        wf = W_final(seq, 2, params=a.params, device=local, shard_world=world, shard_rank=rank, comm_id=obj[0])
    else:
        wf = W_final(seq, 2, params=a.params, device=local)
    for _ in range(a.warmup):
        wf.ccj()
    barrier()
    t0 = time.perf_counter()
    level_ms = fill_ms = 0.0
    for _ in range(a.steps):
        wf.ccj()
        tm = wf.timing()
        level_ms += tm["level4d_ms"]  # the levels' durations: HIP events on the level stream
        fill_ms += tm["fill_ms"]
    elapsed = time.perf_counter() - t0
    barrier()
    # after the timed region: one fold with marker events around every launch (per-kernel-family
    # times for k_iloop / k_diag2d; the markers slow that fold down, so it is not part of `value`)
    wf.set_timing(2)
    wf.ccj()
    tmi = wf.timing()
    il_ms, diag_ms = tmi["iloop_ms"], tmi["diag2d_ms"]
    elapsed = max_over_ranks(elapsed, dist)

    cells = num_cells(a.n)
    wm = (ctypes.c_double * 4)()
    lib().ccj_work_model.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    lib().ccj_work_model(wf._h, wm)
    bytes4d = wm[0]
    ws = (ctypes.c_double * 2)()
    lib().ccj_work_split.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    lib().ccj_work_split(wf._h, ws)
    bytes_il, bytes_lv = ws[0], ws[1]
    nlaunch = max(a.n - 2, 1)
    avg_launch_s = (level_ms / a.steps) / 1e3 / nlaunch
    achieved = (bytes_lv / nlaunch) / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    il_launch_s = il_ms / 1e3 / max(a.n - 6, 1)
    il_achieved = (bytes_il / max(a.n - 6, 1)) / il_launch_s / 1e9 if il_launch_s > 0 else 0.0
    structure, energy = wf.structure, wf.energy
    wf.close()
    # HBM traffic per k_level4d launch, measured with rocprofv3 PMC passes (tools/gpu_profile.sh ->
    # tools/make_profiles.py); null when no profile of this configuration is committed
    traffic = None
    tp = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tp) and a.n == 200 and a.seed == 5 and a.params == "Turner04":
        with open(tp) as f:
            tk = json.load(f)["kernels"].get("k_level4d_level")
        if tk:
            traffic = tk["hbm_bytes_per_launch"]

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    sec_per_seq = elapsed / a.steps
    seqs_per_step = 1 if shard else world  # sharded: the whole job folds one sequence per step
    value = job_value(cells, a.steps, elapsed, world, shard)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "DP-cells/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": sec_per_seq * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": f"CCJ pseudoknot MFE fold of a {a.n}-nt random RNA (random.Random({a.seed}), ACGU), "
                               f"rna_{a.params} tables, dangles 2; one fold per GPU per step (batch mode)",
                   "n": a.n, "params": a.params, "cells_per_fold": cells,
                   "parallelism": f"band{world}" if shard else f"batch{world}"},
        "sec_per_sequence": sec_per_seq,
        "sequences_per_s": seqs_per_step * a.steps / elapsed,
        "mfe": energy,
        "structure": structure,
        "breakdown_ms": {"fill_device": fill_ms / a.steps, "level4d_levels": level_ms / a.steps,
                         "iloop_kernels_instrumented_fold": il_ms, "diag2d_kernels_instrumented_fold": diag_ms,
                         "fill_instrumented_fold": tmi["fill_ms"]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
                     "algorithmic_bytes_per_launch": bytes_lv / nlaunch,
                     "kernel": "k_level4d (one level = k_level4d + k_level4d_lead on the split-sharing "
                               "levels, in order on one stream; duration = the level's time on that stream, "
                               "HIP events over the timed region)",
                     "launches_per_fold": nlaunch,
                     "avg_launch_us": avg_launch_s * 1e6, "algorithmic_bytes_per_fold": bytes_lv},
        "roofline_iloop": {"bound": "hbm", "achieved": il_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": il_achieved / HBM_PEAK_GBS, "kernel": "k_iloop (one instrumented fold after "
                                                                         "the timed region)",
                           "launches_per_fold": max(a.n - 6, 1), "avg_launch_us": il_launch_s * 1e6,
                           "algorithmic_bytes_per_fold": bytes_il},
    }
    if world == 1 and not a.no_cpu_baseline:
        cb = cpu_baseline(a.cpu_sample_n)
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu_baseline_cells_per_s"] = value / cb["value"]
    out["reference_cpu_n200_s"] = 1341.5  # measured reference fold, 1 Xeon core
    out["speedup_vs_reference_n200"] = 1341.5 / sec_per_seq if a.n == 200 else None
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
