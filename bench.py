#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X CCJ engine (BASELINE.json metric/config 3).

One "step" = one complete CCJ MFE fold of one sequence: ccj_reset (the per-sequence setup the
reference does in W_final::W_final, W_final.cc:20-56: encoding, pair/hairpin/stack tables, the
interior-loop work lists) followed by the GPU fill of all 22 four-dimensional gap matrices and the
2-D matrices, exterior W, traceback and bracket emission (on the GPU; the structure string and MFE
are copied back) — everything W_final(seq, 2).ccj() does in the reference.  The default sequence
is the 200-nt headline RNA (random.Random(5), ACGU) with rna_Turner04 tables and dangles 2.
Inputs are resident before the timed region: the contexts (HBM allocations, ccj_create) are
created during setup and their time is reported as `create_ms`.  With `--inflight 2` a batch of
folds is pipelined over two contexts per GPU (fold k+1's fill starts when fold k's fill ends, beside
fold k's W + traceback; measured slower, so the default is 1).  Every fold is complete (ccj_wait)
before the clock stops, and the barrier + wall clock around the K steps brackets finished GPU work.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 200] [--seed 5] [--params Turner04]
                    [--distinct] [--shard]

Multi-GPU (one process per GPU):
  * launched by torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE set), or
  * `--gpus N` alone: this script starts the N rank processes itself before anything touches the
    GPU (fresh children with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) and exits with their status.
Batch mode (default, weak scaling, no data-path collective): rank r folds seed + r (so
`--n 400 --seed 6 --gpus 8` is BASELINE config 5, seeds 6..13); with --distinct, step k of rank r
folds seed + r + N*k instead, a new sequence every step.  --shard band-shards ONE sequence over
all ranks (RCCL all-gather per level, strong scaling).  The barrier and the
max-over-ranks time use torch.distributed (gloo).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import random
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sec/sequence + DP-cells/s at n=200 (Turner04), 1/2/4/8 GPU vs CPU ref"
PF_METRIC = "partition-function DP-cells/s (W_final_pf::ccj_pf, SURVEY 8 f4)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec
REF_N200_S = 1341.5    # BASELINE.md / SURVEY.md §6: reference fold of the headline sequence, 1 Xeon core


def rseq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


def num_cells(n):
    """C(n+1,4), the 4-D DP cells of one fold; same as ccj_amd.num_cells."""
    if n < 3:
        return 0
    m = n + 1
    return m * (m - 1) * (m - 2) * (m - 3) // 24


def footprint_gb(n, sharded=False):
    """Device memory of one context: 4-D matrices (11 stored per level, all 22 when
    band-sharded), loop records, interior-loop copies, candidate lists, the sharing ring and the 2-D
    tables."""
    cells = num_cells(n)
    nm4 = 22 if sharded else 11
    maxc = max(((t + 1) * ((n - t - 2) * (n - t - 1) // 2) for t in range(max(n - 2, 1))), default=0)
    pmx = 2 * sum((n - t - 2) * n * (t + 1) for t in range(max(n - 2, 0)))
    plane = (n + 1) * (n + 2)
    return (2 * nm4 * cells + 44 * cells + 4 * cells + pmx + 320 * maxc + 2 * 841 * plane + 2 * 848 * 8 * plane) / 1e9


def rank_seed(base, rank, world, step, distinct):
    """Seed of the sequence rank folds at a step: seed + rank (batch), or a new one every step."""
    return base + rank + (world * step if distinct else 0)


def max_over_ranks(elapsed, dist):
    """The job's time: the slowest rank's wall clock over the timed steps (gloo all-reduce MAX)."""
    if dist is None:
        return elapsed
    import torch
    tt = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def sum_over_ranks(x, dist):
    if dist is None:
        return x
    import torch
    tt = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.SUM)
    return float(tt.item())


def job_value(cells, steps, elapsed, world, shard):
    """Whole-job DP-cells/s: batch mode folds one sequence per rank per step, band sharding one
    sequence per step over all ranks."""
    seqs_per_step = 1 if shard else world
    return seqs_per_step * steps * cells / elapsed


def share_comm_id(rank, dist, make_id):
    """The band-sharded fold's RCCL unique id: rank 0 makes it (ccj_amd.comm_unique_id), every rank
    receives the same 128 bytes over torch.distributed (gloo) before any rank calls ccj_comm_init."""
    obj = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """Start n rank processes of this script (before any GPU call in this process) and return the
    worst exit status.  Each child gets its own RANK/LOCAL_RANK and the shared rendezvous."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def host_cores():
    """CPU threads this process may use (the GPU box's share, not the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = int(os.environ.get("CCJ_CPU_BASELINE_CORES", "16"))  # gpurun: 16 CPUs per GPU
    return max(1, min(n, cap))


def ref_allcores_n200():
    """The committed all-cores reference measurement at n=200 (profiles/r*_ref_allcores_n200.json,
    written from tools/ref_allcores.py's output), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_ref_allcores_n200.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return {"value": d["value"], "unit": d["unit"], "cores": d["cores"], "wall_s": d["wall_s"],
            "per_process_seconds": d["per_process_seconds"], "kind": "reference",
            "source": "profiles/" + os.path.basename(files[-1]),
            "sample": f"{d['cores']} concurrent reference folds of n=200 random RNAs (seeds "
                      f"{d['seeds'][0]}..{d['seeds'][1]}, Turner04) on the GPU box's host"}


def _ref_fold_cmd(drv, blob, seq):
    return [drv, "fold", "--blob", blob, "--time", seq]


def cpu_baseline(n_sample=110, seed=3, params="Turner04", cores=None):
    """Reference CPU CCJ (oracle/_ref/ref_driver, compiled from the reference sources) on a bounded
    sample of the same workload, at all host cores.  The reference is single-threaded
    (CCJ.cc:44-49 folds one sequence on one thread), so its all-cores form is k concurrent
    processes, each folding its own n_sample-nt sequence (seeds seed..seed+k-1); value = the
    aggregate DP-cells/s of the k folds over the wall time of the slowest.  The first process's own
    time is also reported as the 1-core figure.  Falls back to our C restatement
    (oracle/ccj_oracle.c, level-parallel over the same k threads) when the reference is not built."""
    k = cores or host_cores()
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    blob = os.path.join(ROOT, "ccj_amd", "params", params + ".ccjp")
    cells = num_cells(n_sample)
    if os.path.exists(drv):
        t0 = time.perf_counter()
        procs = [subprocess.Popen(_ref_fold_cmd(drv, blob, rseq(seed + r, n_sample)), stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True) for r in range(k)]
        outs = [p.communicate(timeout=900) for p in procs]
        wall = time.perf_counter() - t0
        per = []
        for p, (_, err) in zip(procs, outs):
            if p.returncode == 0 and "TIME" in err:
                per.append(float(err.split("TIME")[1].split()[0]))
        if len(per) == k:
            return {"value": k * cells / wall, "unit": "DP-cells/s", "cores": k, "kind": "reference",
                    "seconds": wall, "n": n_sample,
                    "single_core": {"value": cells / per[0], "seconds": per[0], "cores": 1},
                    "per_process_seconds": {"min": min(per), "max": max(per)},
                    "sample": f"{k} concurrent full reference folds (W_final::ccj, incl. its constructor), one per "
                              f"host core, of {n_sample}-nt random RNAs (seeds {seed}..{seed + k - 1}, {params}, "
                              f"{cells} cells each); the reference is single-threaded, so k processes are its "
                              f"all-cores form.  An n={n_sample} sample, not the n=200 headline: the reference's "
                              f"cells/s falls with n (see reference_n200_cells_per_s)"}
    from tests.oracle_lib import OracleFold
    with open(blob, "rb") as f:
        b = f.read()
    t0 = time.perf_counter()
    o = OracleFold(rseq(seed, n_sample), b, 2, 0, threads=k)
    t = time.perf_counter() - t0
    o.close()
    return {"value": cells / t, "unit": "DP-cells/s", "cores": k, "kind": "port", "seconds": t, "n": n_sample,
            "sample": f"C restatement fill (level-parallel, {k} threads) of a {n_sample}-nt random RNA "
                      f"(seed {seed}, {params})"}


def pf_cpu_baseline(n_sample=80, seed=3, cores=None):
    """The reference's partition function (oracle/_ref/pf_driver: part_func.cc built from the reference
    sources with -ffp-contract=off, Turner 2004 defaults, dangles 2) on k concurrent processes, one
    n_sample-nt fold each (the reference is single-threaded); value = aggregate 4-D cells/s over the
    slowest process's wall time.  None when the driver is not built."""
    k = cores or host_cores()
    drv = os.path.join(ROOT, "oracle", "_ref", "pf_driver")
    if not os.path.exists(drv):
        return None
    cells = num_cells(n_sample)
    t0 = time.perf_counter()
    procs = [subprocess.Popen([drv, rseq(seed + r, n_sample), "-d", "2"], stdout=subprocess.DEVNULL,
                              stderr=subprocess.DEVNULL) for r in range(k)]
    rcs = [p.wait(timeout=900) for p in procs]
    wall = time.perf_counter() - t0
    if any(rcs):
        return None
    return {"value": k * cells / wall, "unit": "DP-cells/s", "cores": k, "kind": "reference", "seconds": wall,
            "n": n_sample,
            "sample": f"{k} concurrent reference partition-function folds (W_final_pf::ccj_pf incl. its "
                      f"constructor) of {n_sample}-nt random RNAs (seeds {seed}..{seed + k - 1}, Turner 2004, "
                      f"dangles 2), one per host core; O(n^5), so its cells/s falls with n"}


def pf_bench(a, rank, world, dist, barrier, dev=0):
    """--pf: one step = ccj_pf() (the whole fill + W + energy) of the rank's sequence on a context
    created before the timed region.  Replicas only: the PF path has no sharded form, so --gpus N
    runs N independent folds (seed + rank), weak scaling."""
    from ccj_amd import W_final_pf
    seq = rseq(a.seed + rank, a.n)
    t_c = time.perf_counter()
    pf = W_final_pf(seq, dangle=2, params=a.params, device=dev)
    create_ms = (time.perf_counter() - t_c) * 1e3
    for _ in range(a.warmup):
        pf.ccj_pf()
    barrier()
    fill_ms = 0.0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        e = pf.ccj_pf()
        fill_ms += pf.fill_ms()
    elapsed = time.perf_counter() - t0
    barrier()
    elapsed = max_over_ranks(elapsed, dist)
    # after the timed region: one fill with an event pair around every launch (per-family durations)
    pf.set_timing(True)
    pf.ccj_pf()
    kms = pf.kernel_ms()
    pf.set_timing(False)
    work = pf.work_model()
    pf.close()
    if rank != 0:
        return
    cells = num_cells(a.n)
    nl = {"k_pf_iloop": max(a.n - 2, 1), "k_pf_level": max(a.n - 2, 1), "k_pf_pterm": max(a.n - 3, 1),
          "k_pf_ppush": max(a.n - 3, 1), "k_pf_diag": a.n}

    # HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over this workload
    # (tools/gpu_pf_prof.sh -> tools/make_profiles.py --pf), when committed
    tj, tname = find_traffic(a.n, a.seed, a.params, pf=True) if world == 1 else (None, None)

    def roof(k):
        ms = kms[k]
        gbs = work[k] / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        avg_s = ms / 1e3 / nl[k]
        tk = tj["kernels"].get(k) if tj else None
        traffic = tk["hbm_bytes_per_launch"] if tk else None
        return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": f"profiles/{tname}" if tk else None,
                "frac_counter": traffic / avg_s / 1e9 / HBM_PEAK_GBS if traffic and avg_s > 0 else None,
                "kernel": k, "launches_per_fold": nl[k], "avg_launch_us": avg_s * 1e6,
                "algorithmic_bytes_per_fold": work[k], "kernel_ms_per_fold": ms}
    dom = max(kms, key=kms.get)
    out = {
        "metric": PF_METRIC, "value": cells * world * a.steps / elapsed, "unit": "DP-cells/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64+int32", "data": "synthetic",
        "config": {"workload": f"CCJ partition function (W_final_pf::ccj_pf: fill of the 21 int32 4-D and 8 double "
                               f"2-D matrices, W, energy; bit-identical to part_func.cc) of a {a.n}-nt random "
                               f"ACGU RNA per GPU (seed {a.seed}+rank), rna_{a.params}, dangles 2; replicas",
                   "n": a.n, "seed": a.seed, "params": a.params, "cells_per_fold": cells,
                   "parallelism": f"replicas{world}"},
        "sec_per_sequence": elapsed / a.steps, "nt_per_s": a.n * world * a.steps / elapsed,
        "fill_ms": fill_ms / a.steps, "create_ms": create_ms, "energy": e,
        "kernel_ms_instrumented_fold": kms,
        "roofline": roof(dom),
        "roofline_by_kernel": {k: roof(k) for k in kms},
    }
    if world == 1 and not a.no_cpu_baseline:
        cb = pf_cpu_baseline(a.pf_cpu_sample_n, cores=a.cpu_cores)
        if cb:
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu_baseline_cells_per_s"] = out["value"] / cb["value"]
    print(json.dumps(out), flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--params", default="Turner04")
    ap.add_argument("--distinct", action="store_true",
                    help="fold a new sequence every step (seed + rank + world*step) instead of the rank's own")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-n", type=int, default=110)
    ap.add_argument("--cpu-cores", type=int, default=None,
                    help="concurrent reference folds in cpu_baseline (default: this process's CPUs, at most 16)")
    ap.add_argument("--shard", action="store_true",
                    help="band-shard ONE sequence over all ranks (RCCL all-gather per level, strong scaling) "
                         "instead of one sequence per GPU")
    ap.add_argument("--inflight", type=int, default=None,
                    help="folds in flight per GPU (contexts): 2 overlaps one fold's traceback and the next "
                         "sequence's setup with the next fill (default 1, measured faster; 2 only when two "
                         "contexts fit in HBM, never band-sharded)")
    ap.add_argument("--pf", action="store_true",
                    help="the partition-function path (W_final_pf::ccj_pf, SURVEY §8 f4) instead of the MFE "
                         "fold: one step = one PF fill + W of the rank's sequence (replicas, no collective)")
    ap.add_argument("--pf-cpu-sample-n", type=int, default=80)
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the rank launch, barrier and max-over-ranks accounting only (tests)")
    return ap.parse_args(argv)


def find_traffic(n, seed, params, pf=False):
    """The committed rocprofv3 FETCH_SIZE/WRITE_SIZE summary (tools/make_profiles.py) of this exact
    workload: profiles/traffic*.json whose "config" is (n, seed, params) and whose "pf" flag is pf;
    the untagged profiles/traffic.json of rounds 1-3 is the headline n=200 seed 5 Turner04 fold."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic*.json"))):
        with open(path) as f:
            tj = json.load(f)
        cfg = tj.get("config", {"n": 200, "seed": 5, "params": "Turner04"})
        if (cfg.get("n"), cfg.get("seed"), cfg.get("params")) == (n, seed, params) and bool(tj.get("pf")) == pf:
            return tj, os.path.basename(path)
    return None, None


def rank_device(local):
    """The GPU of this rank: LOCAL_RANK when every GPU of the node is visible to each rank (the
    driver's torch.distributed.run launch), else LOCAL_RANK modulo the visible devices (one GPU per
    rank through HIP_VISIBLE_DEVICES, or a rehearsal of N ranks on a 1-GPU box).  Counting devices
    does not initialise the GPU on this image."""
    if local == 0:
        return 0  # (no torch import on the single-rank path)
    try:
        import torch
        n = torch.cuda.device_count()
    except Exception:
        n = 0
    if n <= 0:
        # no torch count: the visible-device list, else device 0 (never an index past what the
        # rank can see, e.g. LOCAL_RANK 3 with one GPU per rank)
        vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") or ""
        n = len([v for v in vis.split(",") if v.strip()])
    return local % n if n > 0 else 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if a.gpus is not None and a.gpus > 1 and env_world is None:
        # one process per GPU: start them now, before this process makes any GPU call
        sys.exit(spawn_ranks(a.gpus, argv))
    world = int(env_world or "1")
    if a.gpus is not None and a.gpus != world:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = rank_device(local) if not a.dry_run else local
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    shard = a.shard and world > 1
    cells = num_cells(a.n)
    rank_devs = [dev]
    if dist is not None:  # the rank -> GPU mapping goes on the line, so a mis-mapped rank is visible
        rank_devs = [None] * world
        dist.all_gather_object(rank_devs, dev)

    def seq_at(step):
        return rseq(a.seed if shard else rank_seed(a.seed, rank, world, step, a.distinct), a.n)

    if a.dry_run:
        comm_ok = None
        if shard:  # the comm-id hand-off of the sharded path, with a stand-in id (no RCCL, no GPU)
            cid = share_comm_id(rank, dist, lambda: os.urandom(128))
            ids = [None] * world
            dist.all_gather_object(ids, cid)
            comm_ok = len(cid) == 128 and all(x == cid for x in ids)
        barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            time.sleep(0.001)
        elapsed = max_over_ranks(time.perf_counter() - t0, dist)
        ranks = int(sum_over_ranks(1.0, dist))
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": job_value(cells, a.steps, elapsed, world, shard),
                              "unit": "DP-cells/s", "n_gpus": world, "ranks_reported": ranks, "steps": a.steps,
                              "warmup": a.warmup, "dry_run": True, "shard": shard, "comm_id_agreed": comm_ok,
                              "seeds": [rank_seed(a.seed, r, world, 0, a.distinct) for r in range(world)]}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    if a.pf:
        pf_bench(a, rank, world, dist, barrier, dev)
        if dist is not None:
            dist.destroy_process_group()
        return

    import ctypes
    from ccj_amd import W_final, lib, comm_unique_id

    # 1 by default: with 2 contexts the fill measured 3 ms slower (their streams share
    # the 4 hardware queues, so one fold's one-wave traceback holds up the other's level launches)
    inflight = a.inflight if a.inflight is not None else 1
    if 2 * footprint_gb(a.n) > 200:
        inflight = 1
    inflight = 1 if shard else max(1, min(2, inflight))
    t_c = time.perf_counter()
    if shard:
        cid = share_comm_id(rank, dist, comm_unique_id)
        ctxs = [W_final(seq_at(0), 2, params=a.params, device=dev, shard_world=world, shard_rank=rank, comm_id=cid)]
    else:
        ctxs = [W_final(seq_at(0), 2, params=a.params, device=dev) for _ in range(inflight)]
    create_ms = (time.perf_counter() - t_c) * 1e3 / len(ctxs)

    def run_steps(nsteps, acc):
        """nsteps folds, pipelined over the contexts: while fold k's fill (then its W + traceback,
        one wave) runs on context k % inflight, the host resets the next context to sequence k+1 and
        enqueues its fill, so the traceback and the setup hide under the next fill."""
        def start(k):
            wf = ctxs[k % len(ctxs)]
            tr = time.perf_counter()
            wf.reset(seq_at(k))  # per-sequence setup, inside the timed region
            acc["reset_s"] += time.perf_counter() - tr
            # the fill of k starts when fill k-1 has ended; k-1's traceback runs beside it
            wf.fill_async(after=ctxs[(k - 1) % len(ctxs)] if len(ctxs) > 1 and k > 0 else None)
        start(0)
        for k in range(nsteps):
            if len(ctxs) > 1 and k + 1 < nsteps:
                start(k + 1)
            wf = ctxs[k % len(ctxs)]
            wf.wait()
            tm = wf.timing()
            acc["level_ms"] += tm["level4d_ms"]  # the levels' durations: HIP events on the level stream
            acc["fill_ms"] += tm["fill_ms"]
            acc["last"] = wf
            if len(ctxs) == 1 and k + 1 < nsteps:
                start(k + 1)

    run_steps(a.warmup, {"reset_s": 0.0, "level_ms": 0.0, "fill_ms": 0.0}) if a.warmup > 0 else None
    barrier()
    acc = {"reset_s": 0.0, "level_ms": 0.0, "fill_ms": 0.0, "last": ctxs[0]}
    t0 = time.perf_counter()
    run_steps(a.steps, acc)
    elapsed = time.perf_counter() - t0
    barrier()
    reset_s, level_ms, fill_ms = acc["reset_s"], acc["level_ms"], acc["fill_ms"]
    structure, energy = acc["last"].structure, acc["last"].energy
    wf = ctxs[0]
    # after the timed region: one fold with marker events around every launch (per-kernel-family
    # times for the interior loops (k_iloop) / k_diag2d; the
    # markers slow that fold down, so it is not part of `value`)
    wf.set_timing(2)
    wf.ccj()
    tmi = wf.timing()
    il_ms, diag_ms, pp_ms = tmi["iloop_ms"], tmi["diag2d_ms"], tmi["ppush_ms"]
    elapsed = max_over_ranks(elapsed, dist)

    wm = (ctypes.c_double * 4)()
    lib().ccj_work_model.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    lib().ccj_work_model(wf._h, wm)
    ws = (ctypes.c_double * 2)()
    lib().ccj_work_split.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    lib().ccj_work_split(wf._h, ws)
    bytes_il, bytes_lv = ws[0], ws[1]
    nlaunch = max(a.n - 2, 1)
    avg_launch_s = (level_ms / a.steps) / 1e3 / nlaunch
    achieved = (bytes_lv / nlaunch) / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    il_launch_s = il_ms / 1e3 / max(a.n - 6, 1)
    il_achieved = (bytes_il / max(a.n - 6, 1)) / il_launch_s / 1e9 if il_launch_s > 0 else 0.0
    for w in ctxs:
        w.close()
    # HBM traffic per level, measured with rocprofv3 PMC passes over this same command
    # (tools/gpu_profile.sh -> tools/make_profiles.py -> profiles/traffic.json); null when no
    # profile of this configuration is committed (it is not measured inside this run)
    traffic = traffic_src = None
    il_kernel = "k_iloop"
    il_traffic = None
    tj, tname = find_traffic(a.n, a.seed, a.params) if world == 1 or not shard else (None, None)
    side_traffic = {}  # kernel -> (counter bytes per launch, launches per fold)
    fill_counter_bytes = None
    if tj:
        tk = tj["kernels"].get("k_level4d_level")
        if tk:
            traffic = tk["hbm_bytes_per_launch"]
            traffic_src = f"profiles/{tname} (" + tj.get("source", "rocprofv3 PMC passes") + ")"
        ti = tj["kernels"].get(il_kernel)
        if ti:
            il_traffic = ti["hbm_bytes_per_launch"]
        if tk:
            folds = tk["launches"] / nlaunch  # the profiled command's folds
            for kn, kv in tj["kernels"].items():
                if kn.startswith("k_level4d"):
                    continue  # the level chain: k_level4d_level (= k_level4d + k_level4d_lead), counted below
                side_traffic[kn.split("<")[0]] = (kv["hbm_bytes_per_launch"], kv["launches"] / folds)
            fill_counter_bytes = sum(b * l for b, l in side_traffic.values())

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    sec_per_step = elapsed / a.steps
    seqs_per_step = 1 if shard else world  # sharded: the whole job folds one sequence per step
    value = job_value(cells, a.steps, elapsed, world, shard)
    if shard:
        wl = f"one {a.n}-nt sequence per step band-sharded over {world} GPUs"
    elif a.distinct:
        wl = f"a new {a.n}-nt sequence per GPU per step (seed + rank + {world}*step)"
    else:
        wl = f"one {a.n}-nt sequence per GPU per step (rank r: seed {a.seed}+r)"
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "DP-cells/s",
        "n_gpus": world,
        "rank_devices": rank_devs,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": sec_per_step * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": f"CCJ pseudoknot MFE fold (ccj_reset + fill + W + traceback) of random ACGU RNA "
                               f"(random.Random(seed)), rna_{a.params} tables, dangles 2; {wl}; "
                               f"{len(ctxs)} fold(s) in flight per GPU",
                   "n": a.n, "seed": a.seed, "params": a.params, "cells_per_fold": cells,
                   "parallelism": f"band{world}" if shard else f"batch{world}"},
        "sec_per_sequence": sec_per_step,  # latency of one fold (every rank folds one per step in batch mode)
        "sequences_per_s": seqs_per_step * a.steps / elapsed,
        "nt_per_s": a.n * seqs_per_step * a.steps / elapsed,
        "create_ms": create_ms,
        "setup_ms": reset_s / a.steps * 1e3,
        "inflight": len(ctxs),
        "mfe": energy,
        "structure": structure,
        "rank0_last_seq_seed": a.seed if shard else rank_seed(a.seed, 0, world, a.steps - 1, a.distinct),
        "breakdown_ms": {"setup_reset": reset_s / a.steps * 1e3, "fill_device": fill_ms / a.steps,
                         "level4d_levels": level_ms / a.steps,
                         "iloop_kernels_instrumented_fold": il_ms, "diag2d_kernels_instrumented_fold": diag_ms,
                         "ppush_kernels_instrumented_fold": pp_ms,
                         "fill_instrumented_fold": tmi["fill_ms"]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": bytes_lv / nlaunch,
                     "kernel": "k_level4d (one level = k_level4d + k_level4d_lead on the split-sharing "
                               "levels, in order on one stream; duration = the level's time on that stream, "
                               "HIP events over the timed region)",
                     "launches_per_fold": nlaunch,
                     "avg_launch_us": avg_launch_s * 1e6, "algorithmic_bytes_per_fold": bytes_lv,
                     # the measured HBM bytes (FETCH_SIZE + WRITE_SIZE, rocprofv3 PMC) over the same level
                     # duration: the counter-based bandwidth fraction beside the algorithmic one
                     "frac_counter": (traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS) if traffic and avg_launch_s > 0 else None,
                     "achieved_counter_gbs": (traffic / avg_launch_s / 1e9) if traffic and avg_launch_s > 0 else None},
        "roofline_iloop": {"bound": "hbm", "achieved": il_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": il_achieved / HBM_PEAK_GBS,
                           "kernel": il_kernel + " (one instrumented fold after the timed region)",
                           "launches_per_fold": max(a.n - 6, 1), "avg_launch_us": il_launch_s * 1e6,
                           "algorithmic_bytes_per_fold": bytes_il, "traffic": il_traffic, "traffic_unit": "bytes/launch",
                           "frac_counter": (il_traffic / il_launch_s / 1e9 / HBM_PEAK_GBS) if il_traffic and il_launch_s > 0 else None},
    }
    # the side kernels in the fill (instrumented fold: marker events around every launch, so these
    # are in-fill durations with the level chain beside them, not standalone figures)
    pp_n = side_traffic.get("k_ppush", (None, max(a.n - 3, 1)))[1]
    pp_launch_s = pp_ms / 1e3 / pp_n if pp_ms else 0.0
    pp_tr = side_traffic.get("k_ppush", (None, 0))[0]
    out["roofline_ppush"] = {
        "bound": "hbm", "kernel": "k_ppush (P terms pushed by level; one instrumented fold after the timed region)",
        "launches_per_fold": pp_n, "avg_launch_us": pp_launch_s * 1e6, "algorithmic_bytes_per_fold": wm[1],
        "achieved": (wm[1] / pp_n) / pp_launch_s / 1e9 if pp_launch_s > 0 else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": (wm[1] / pp_n) / pp_launch_s / 1e9 / HBM_PEAK_GBS if pp_launch_s > 0 else None,
        "traffic": pp_tr, "traffic_unit": "bytes/launch",
        "frac_counter": pp_tr / pp_launch_s / 1e9 / HBM_PEAK_GBS if pp_tr and pp_launch_s > 0 else None}
    dg_n = side_traffic.get("k_diag2d", (None, a.n))[1]
    dg_launch_s = diag_ms / 1e3 / dg_n if diag_ms else 0.0
    dg_tr = side_traffic.get("k_diag2d", (None, 0))[0]
    out["roofline_diag2d"] = {
        "bound": "latency", "kernel": "k_diag2d (2-D spans, cache-resident; one instrumented fold)",
        "launches_per_fold": dg_n, "avg_launch_us": dg_launch_s * 1e6, "traffic": dg_tr, "traffic_unit": "bytes/launch",
        "frac_counter": dg_tr / dg_launch_s / 1e9 / HBM_PEAK_GBS if dg_tr and dg_launch_s > 0 else None}
    if fill_counter_bytes is not None and traffic:
        fb = fill_counter_bytes + traffic * nlaunch
        out["fill_counter"] = {"hbm_bytes_per_fold": fb, "fill_ms": fill_ms / a.steps,
                               "gbs": fb / (fill_ms / a.steps / 1e3) / 1e9,
                               "frac": fb / (fill_ms / a.steps / 1e3) / 1e9 / HBM_PEAK_GBS,
                               "source": traffic_src}
    # the algorithmic model charges every operand read (split-sharing and the caches serve many of
    # them); when its bytes per fold exceed what HBM could move in the fold's time it is an
    # effective-bandwidth figure, not an HBM fraction: say so on the line
    alg_step_gbs = (bytes_lv + bytes_il) / sec_per_step / 1e9
    out["algorithmic_gbs_per_step"] = alg_step_gbs
    if alg_step_gbs > HBM_PEAK_GBS or out["roofline"]["frac"] > 1.0:
        out["roofline"]["note"] = ("algorithmic bytes exceed the HBM peak: frac is an effective (cache-served) "
                                   "bandwidth, not an HBM fraction; see frac_counter")
    if world == 1 and not a.no_cpu_baseline:
        cb = cpu_baseline(a.cpu_sample_n, cores=a.cpu_cores)
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu_baseline_cells_per_s"] = value / cb["value"]
    # the reference at the headline size itself (measured in the survey container, not on the box)
    out["reference_cpu_n200_s"] = REF_N200_S
    out["reference_n200_cells_per_s"] = num_cells(200) / REF_N200_S
    out["speedup_vs_reference_n200"] = REF_N200_S / sec_per_step if a.n == 200 else None
    # the reference at the headline size on ALL host cores of a GPU box (16 concurrent n=200 folds,
    # tools/ref_allcores.py; 12-15 min of CPU time, so measured once and committed, not per run)
    ra = ref_allcores_n200()
    if ra and a.n == 200:
        out["reference_n200_allcores"] = ra
        out["speedup_vs_reference_n200_allcores"] = value / ra["value"]
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
