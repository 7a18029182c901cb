"""Band sharding of one sequence — host logic, on CPU.

* ccj_shard_range partitions every level's a-blocks into contiguous per-rank ranges, and
  ccj_level_layout pads each matrix of the level to world equal chunks, so rank r's blocks are
  exactly chunk r of every matrix: an in-place all-gather per matrix rebuilds the whole level.
* world-size-2 gloo run: each rank writes only its own blocks of every level (cell values from the
  C oracle, which is the checker here), the chunks are all-gathered as the RCCL path does on the
  GPU, and the gathered levels must equal the levels written by one process.
"""
import os
import random

import numpy as np
import pytest

from tests.oracle_lib import OracleFold, blob

NMAT4 = 22


def _rseq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


@pytest.mark.parametrize("n", [7, 33, 200])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_ranges_partition_levels(n, world):
    from ccj_amd import level_layout, shard_range
    for t in range(max(n - 2, 1)):
        C, M = level_layout(n, t, world)
        B = -(-(t + 1) // world)
        assert C == (t + 1) * M if world == 1 else C == B * world * M
        nxt = 0
        for r in range(world):
            lo, end = shard_range(n, t, world, r)
            assert lo == min(nxt, t + 1) and lo <= end <= t + 1
            if world > 1:
                assert end - lo <= B and lo == min(r * B, t + 1)  # chunk r of C holds blocks [rB, (r+1)B)
            nxt = end
        assert nxt == t + 1


def _level_buffer(n, t, world, fold, ranks):
    """22 matrices of level t in the (padded) device layout, cells of the given ranks' blocks only."""
    from ccj_amd import level_layout, shard_range
    C, M = level_layout(n, t, world)
    m = n - t - 2
    buf = np.zeros(NMAT4 * C, dtype=np.int16)
    for r in ranks:
        lo, end = shard_range(n, t, world, r)
        for a in range(lo, end):
            b = t - a
            for h in range(m):
                for i in range(1, m - h + 1):
                    j, k = i + a, i + a + h + 2
                    l = k + b
                    off = a * M + h * m - h * (h - 1) // 2 + (i - 1)
                    for x in range(NMAT4):
                        buf[x * C + off] = fold.get4(x, i, j, k, l)
    return buf, C


def _gloo_rank(rank, world, port, n, seq, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _gloo_body(rank, world, n, seq, q, torch, dist)
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _gloo_body(rank, world, n, seq, q, torch, dist):
    if True:
        fold = OracleFold(seq, blob("Turner04"), 2, 0)
        ok = True
        for t in range(n - 2):
            mine, C = _level_buffer(n, t, world, fold, [rank])
            chunk = C // world
            gathered = np.array(mine)
            for x in range(NMAT4):
                # bytes, as the RCCL path sends them: ncclAllGather(base + rank*chunk, base, 2*chunk, ncclInt8)
                own = torch.from_numpy(mine[x * C + rank * chunk: x * C + (rank + 1) * chunk].copy()).view(torch.uint8)
                parts = [torch.empty_like(own) for _ in range(world)]
                dist.all_gather(parts, own)
                gathered[x * C: (x + 1) * C] = torch.cat(parts).view(torch.int16).numpy()
            full, _ = _level_buffer(n, t, world, fold, range(world))
            ok &= bool(np.array_equal(gathered, full))
        fold.close()
        q.put((rank, ok))


def test_level_allgather_rebuilds_levels_gloo():
    import torch.multiprocessing as mp
    n, world = 16, 2
    seq = _rseq(11, n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random(os.getpid()).randrange(2000)
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, n, seq, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
