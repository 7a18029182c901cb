"""bench.py's multi-rank accounting on CPU (gloo, world size 2): the job time is the slowest rank's
time, and `value` counts every rank's folds in batch mode, one fold per step when band-sharded."""
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, bench.max_over_ranks(1.0 + 2.5 * rank, dist)))
    finally:
        dist.destroy_process_group()


def test_max_over_ranks_gloo():
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
