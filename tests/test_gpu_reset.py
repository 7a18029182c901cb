"""ccj_reset (-m gpu): one context folds a batch of equal-length sequences, rebuilding only the
per-sequence tables and interior-loop work lists.  Every fold after a reset must equal a fresh
context's fold of the same sequence and the C oracle, bit for bit, including when the new
sequence has more pairable positions (larger work lists) than the one the context was built for.
"""
import random

import pytest

from tests.oracle_lib import OracleFold, blob

pytestmark = pytest.mark.gpu


def _rseq(seed, n, alphabet="ACGU"):
    r = random.Random(seed)
    return "".join(r.choice(alphabet) for _ in range(n))


@pytest.mark.parametrize("params", ["Turner04", "DirksPierce09"])
def test_reset_batch_matches_oracle(params):
    from ccj_amd import W_final
    n = 48
    # AU-poor start, then GC-rich (more pairs: the work-list buffer must grow), then mixed
    seqs = [_rseq(1, n, "AAAAUC"), _rseq(2, n, "GGCCAU"), _rseq(3, n), _rseq(4, n, "GCGU")]
    wf = W_final(seqs[0], 2, params=params)
    try:
        for s in seqs:
            wf.reset(s)
            e = wf.ccj()
            o = OracleFold(s, blob(params), 2, 0)
            try:
                assert wf.hashes() == o.hashes()
                assert e == o.W(n) / 100.0
            finally:
                o.close()
    finally:
        wf.close()


def _outcome(wf):
    from ccj_amd import BacktrackExit
    try:
        return ("ok", wf.ccj(), wf.structure, wf.stdout_msgs)
    except BacktrackExit as ex:
        return ("exit", ex.exit_code, ex.msg, ex.stdout)


def test_reset_equals_fresh_context_at_n120():
    from ccj_amd import W_final
    a, b = _rseq(11, 120), _rseq(12, 120)
    wf = W_final(a, 2, params="Turner04")
    fresh = W_final(b, 2, params="Turner04")
    try:
        _outcome(wf)
        wf.reset(b)
        assert _outcome(wf) == _outcome(fresh)  # (some random inputs hit the reference's backtrack exits)
        assert wf.hashes() == fresh.hashes()
    finally:
        wf.close()
        fresh.close()


def test_reset_rejects_other_lengths():
    from ccj_amd import W_final, CCJError
    wf = W_final(_rseq(5, 30), 2, params="Turner04")
    try:
        with pytest.raises(CCJError):
            wf.reset(_rseq(5, 31))
        with pytest.raises(CCJError):
            wf.reset("ACGUX" * 6)
    finally:
        wf.close()


def test_reset_sharded_simulation():
    from ccj_amd import W_final
    a, b = _rseq(21, 64), _rseq(22, 64, "GGCCAU")
    wf = W_final(a, 2, params="Turner04", shard_world=3, shard_simulate=True)
    try:
        _outcome(wf)
        wf.reset(b)
        _outcome(wf)  # W is computed before the traceback, whatever the traceback does
        o = OracleFold(b, blob("Turner04"), 2, 0)
        try:
            assert wf.hashes() == o.hashes()
        finally:
            o.close()
    finally:
        wf.close()


def test_pipelined_contexts_match_synchronous_folds():
    """Two contexts in flight (ccj_fill_async / ccj_wait, as bench.py runs a batch): every fold
    equals the synchronous fold of the same sequence, backtrack exits included."""
    from ccj_amd import W_final, CCJError
    n = 90
    seqs = [_rseq(300 + k, n, "ACGU" if k % 3 else "GGCCAU") for k in range(6)]
    sync = []
    ref = W_final(seqs[0], 2, params="Turner04")
    try:
        for sq in seqs:
            ref.reset(sq)
            sync.append(_outcome(ref))
    finally:
        ref.close()

    def waited(wf):
        from ccj_amd import BacktrackExit
        try:
            return ("ok", wf.wait(), wf.structure, wf.stdout_msgs)
        except BacktrackExit as ex:
            return ("exit", ex.exit_code, ex.msg, ex.stdout)

    ctx = [W_final(seqs[0], 2, params="Turner04"), W_final(seqs[1], 2, params="Turner04")]
    try:
        got = []
        ctx[0].fill_async()
        with pytest.raises(CCJError):
            ctx[0].reset(seqs[2])  # a fold is in flight
        for k in range(len(seqs)):
            if k + 1 < len(seqs):
                nxt = ctx[(k + 1) % 2]
                nxt.reset(seqs[k + 1])
                nxt.fill_async()
            got.append(waited(ctx[k % 2]))
        assert got == sync
    finally:
        for wf in ctx:
            wf.close()
