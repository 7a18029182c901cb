"""Band sharding of one sequence — host logic, on CPU.

* Ownership: a-block a of every level belongs to rank (a // 4) % world, the same rank on every
  level, so a split-sharing leader (a % 4 == 0) and its followers (a+1 .. a+3, on later levels)
  are on one rank; ccj_shard_blocks lists a rank's blocks, and every level's blocks are partitioned.
* Exchange: world-size-2 gloo run.  Each rank packs only its own cells of every level (values from
  the C oracle, which is the checker here) into one slice [matrix][own block][cell] of nmax blocks
  (nmax = the largest rank's block count), the slices are all-gathered as ONE collective per level
  (the RCCL path does the same on the GPU), and unpacking the other ranks' slices must rebuild the
  level exactly as one process writes it.
* 2-D spans: interval i of every span belongs to rank (i-1) % world (k_diag2d); the exchange of
  level t also carries span t (k_dtail_pack / k_dtail_unpack: V, Vt, P, WBP, WPP, WM, WMv, WMp ... of
  the rank's own intervals), and unpacking must give every rank the whole span.
* P terms: each rank pushes only its share of the terms of P(i, i+sigma) (k_ppush outer index
  jo / d-j-1 taken r, r+G, ...), as (value + 2^31) << 32 | first-split key words; the tail of the
  exchange of level sigma-2 carries them and the minimum over the ranks must be the reference's P
  (pseudo_loop.cc:166-179) with its first minimum.
"""
import os
import random

import numpy as np
import pytest

from tests.oracle_lib import OracleFold, blob

NMAT4 = 22
GRP = 4


def _rseq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


def _owner(a, world):
    return (a // GRP) % world


@pytest.mark.parametrize("n", [7, 33, 200])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_blocks_partition_levels(n, world):
    from ccj_amd import level_layout, shard_blocks
    for t in range(max(n - 2, 1)):
        C, M = level_layout(n, t, world)
        assert C == (t + 1) * M  # unpadded for every world
        seen = []
        for r in range(world):
            blocks = shard_blocks(n, t, world, r)
            assert blocks == sorted(blocks)
            assert all(_owner(a, world) == r for a in blocks)
            # a leader's followers a+1..a+3 (the same column on later levels) are on its rank
            for a in blocks:
                if a % GRP == 0:
                    assert all(_owner(a + x, world) == r for x in range(1, GRP))
            seen += blocks
        assert sorted(seen) == list(range(t + 1))
        # balance: ranks differ by at most one group of blocks
        counts = [len(shard_blocks(n, t, world, r)) for r in range(world)]
        assert max(counts) - min(counts) <= GRP


def _cells(n, t, a):
    m = n - t - 2
    b = t - a
    for h in range(m):
        for i in range(1, m - h + 1):
            j, k = i + a, i + a + h + 2
            yield h * m - h * (h - 1) // 2 + (i - 1), (i, j, k, k + b)


def _level(n, t, fold, blocks):
    """22 matrices of level t in the device layout, only the given blocks' cells filled."""
    from ccj_amd import level_layout
    C, M = level_layout(n, t, 1)
    buf = np.zeros(NMAT4 * C, dtype=np.int16)
    for a in blocks:
        for off, (i, j, k, l) in _cells(n, t, a):
            for x in range(NMAT4):
                buf[x * C + a * M + off] = fold.get4(x, i, j, k, l)
    return buf, C, M


def _pack(level, C, M, blocks, nmax):
    """k_pack: slice [x][own index][M] of nmax blocks per matrix."""
    sl = np.zeros(NMAT4 * nmax * M, dtype=np.int16)
    for o, a in enumerate(blocks):
        for x in range(NMAT4):
            sl[(x * nmax + o) * M:(x * nmax + o + 1) * M] = level[x * C + a * M: x * C + (a + 1) * M]
    return sl


def _unpack(level, C, M, slices, world, rank, t, nmax, shard_blocks, n):
    """k_unpack: the other ranks' blocks from their slices."""
    for r in range(world):
        if r == rank:
            continue
        for o, a in enumerate(shard_blocks(n, t, world, r)):
            for x in range(NMAT4):
                level[x * C + a * M: x * C + (a + 1) * M] = slices[r][(x * nmax + o) * M:(x * nmax + o + 1) * M]


def _gloo_rank(rank, world, port, n, seq, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            q.put((rank, _gloo_body(rank, world, n, seq, torch, dist)))
        finally:
            dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))


def p_term_rank(jo, do, ko, sigma, world):
    """The rank that pushes term (j-i, d-i, k-i) of P(i, i+sigma) (k_ppush: part A, t1 = max level,
    by outer index jo; part B, t2 = max level > t1, by outer index d-j-1)."""
    t1 = jo + (ko - do - 1)
    t2 = (do - jo - 1) + (sigma - ko - 1)
    return (jo if t1 >= t2 else do - jo - 1) % world


def _p_partials(fold, n, sigma, world, rank):
    """This rank's (value + 2^31) << 32 | key word of P(i, i+sigma) for i = 0..n (~0: no term)."""
    out = np.full(n + 1, np.iinfo(np.uint64).max, dtype=np.uint64)
    for i in range(1, n - sigma + 1):
        l = i + sigma
        best = None
        for j in range(i, l):
            for d in range(j + 1, l):
                for k in range(d + 1, l):
                    jo, do, ko = j - i, d - i, k - i
                    if p_term_rank(jo, do, ko, sigma, world) != rank:
                        continue
                    v = fold.get4(0, i, j, d + 1, k) + fold.get4(0, j + 1, d, k + 1, l)
                    w = ((v + 2 ** 31) << 32) | ((jo * sigma + do) * sigma + ko)
                    best = w if best is None or w < best else best
        if best is not None:
            out[i] = best
    return out


def _span_tail(fold, n, sigma, world, rank):
    """k_dtail_pack: the 2-D values (oracle get2 ids 0..7) of this rank's intervals of span sigma."""
    tail = np.zeros((8, n + 1), dtype=np.int32)
    for i in range(1, n - sigma + 1):
        if (i - 1) % world == rank:
            tail[:, i] = [fold.get2(x, i, i + sigma) for x in range(8)]
    return tail


def _gloo_body(rank, world, n, seq, torch, dist):
    from ccj_amd import shard_blocks
    fold = OracleFold(seq, blob("Turner04"), 2, 0)
    ok = True
    for t in range(n - 2):
        mine = shard_blocks(n, t, world, rank)
        nmax = max(len(shard_blocks(n, t, world, r)) for r in range(world))
        level, C, M = _level(n, t, fold, mine)
        sig = t + 2  # the P span whose partials ride this exchange (pushed after level t-1)
        tail = _p_partials(fold, n, sig, world, rank) if 1 <= t and sig <= n - 1 else np.zeros(n + 1, np.uint64)
        body = _pack(level, C, M, mine, nmax).view(np.uint8)
        span = _span_tail(fold, n, t, world, rank)
        own = torch.from_numpy(np.concatenate([body, np.zeros((-len(body)) % 8, np.uint8), tail.view(np.uint8),
                                               span.reshape(-1).view(np.uint8)]))
        parts = [torch.empty_like(own) for _ in range(world)]
        dist.all_gather(parts, own)  # ONE collective per level: cells + P tail + span t
        nb = len(body) + (-len(body)) % 8
        slices = [p[:len(body)].numpy().view(np.int16) for p in parts]
        _unpack(level, C, M, slices, world, rank, t, nmax, shard_blocks, n)
        full, _, _ = _level(n, t, fold, range(t + 1))
        ok &= bool(np.array_equal(level, full))
        # k_dtail_unpack: each interval from its owner's slice; the whole span on every rank
        st = nb + 8 * (n + 1)
        spans = [p[st:].numpy().view(np.int32).reshape(8, n + 1) for p in parts]
        for i in range(1, n - t + 1):
            got = spans[(i - 1) % world][:, i]
            ok &= all(int(got[x]) == fold.get2(x, i, i + t) for x in range(8))
        if 1 <= t and sig <= n - 1:
            comb = np.minimum.reduce([p[nb:].numpy().view(np.uint64) for p in parts])
            for i in range(1, n - sig + 1):
                ref = fold.get2(0, i, i + sig)  # reference P (INF+1 when no term)
                got = int(comb[i])
                val = None if got == (1 << 64) - 1 else (got >> 32) - 2 ** 31
                ok &= (val is None and ref == 10000001) or (val == ref)
    fold.close()
    return ok


def test_level_allgather_rebuilds_levels_gloo():
    pytest.importorskip("torch")
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


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_p_term_partition_covers_every_term_once(world):
    """k_ppush's per-rank outer indices r, r+G, ... <= lev partition [0, lev]; every term of P lands
    on exactly one rank."""
    for lev in range(0, 40):
        seen = []
        for r in range(world):
            nout = (lev - r) // world + 1 if r <= lev else 0
            seen += [r + world * x for x in range(nout)]
        assert sorted(seen) == list(range(lev + 1))
    sigma = 12
    for jo in range(sigma):
        for do in range(jo + 1, sigma):
            for ko in range(do + 1, sigma):
                assert 0 <= p_term_rank(jo, do, ko, sigma, world) < world
