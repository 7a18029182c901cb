"""bench.py's multi-rank accounting on CPU (gloo, world size 2): the job time is the slowest rank's
time, and `value` counts every rank's folds in batch mode, one fold per step when band-sharded."""
import multiprocessing as mp
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            q.put((rank, bench.max_over_ranks(1.0 + 2.5 * rank, dist)))
        finally:
            dist.destroy_process_group()
    except Exception as e:  # report to the parent instead of leaving it blocked on the queue
        q.put((rank, repr(e)))


def test_max_over_ranks_gloo():
    pytest.importorskip("torch")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: 3.5, 1: 3.5}


def test_max_over_ranks_single():
    assert bench.max_over_ranks(0.25, None) == 0.25


def test_job_value():
    cells = 65998350
    assert bench.job_value(cells, 5, 0.25, 1, False) == 5 * cells / 0.25
    assert bench.job_value(cells, 5, 0.25, 8, False) == 8 * 5 * cells / 0.25   # batch: weak scaling
    assert bench.job_value(cells, 5, 0.25, 8, True) == 5 * cells / 0.25        # band-sharded: one fold


def test_rank_seeds():
    # batch: rank r folds seed + r (config 5: --seed 6 --gpus 8 -> seeds 6..13); --distinct: new every step
    assert [bench.rank_seed(6, r, 8, 0, False) for r in range(8)] == list(range(6, 14))
    assert bench.rank_seed(6, 3, 8, 5, False) == 9
    assert [bench.rank_seed(5, 1, 2, k, True) for k in range(3)] == [6, 8, 10]


def test_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` with no WORLD_SIZE starts two rank processes itself (gloo, no GPU in
    --dry-run) and rank 0 reports n_gpus 2 with both ranks present."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--dry-run",
                        "--seed", "6"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_reported"] == 2 and out["seeds"] == [6, 7]


def test_gpus_mismatch_fails():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0


def test_shard_dry_run_shares_comm_id():
    """`bench.py --gpus 2 --shard --dry-run`: the sharded path's comm-id hand-off (rank 0 makes the
    128-byte id, every rank receives it over gloo before ccj_comm_init), with no GPU; one fold per
    step for the whole job (strong scaling)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--shard", "--steps", "2",
                        "--dry-run"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["shard"] is True and out["comm_id_agreed"] is True and out["ranks_reported"] == 2
