"""Split-point sharing (ccj_engine.h) on the GPU (-m gpu).

A leader cell scans its whole split range for itself and the next SHARE_R-1 cells of each of its
gap columns; the followers scan only the split points the leader did not see.  Min is
order-independent, so the fill must stay bit-identical to the reference.  By default sharing
covers the unsplit middle levels (n >= ~60); split_target=-1 turns level splitting off so that
sharing covers every level, which exercises leaders, followers and the ring at small n.
"""
import random

import pytest

from tests.oracle_lib import OracleFold, blob, golden

pytestmark = pytest.mark.gpu


def _rseq(seed, n, alphabet="ACGU"):
    r = random.Random(seed)
    return "".join(r.choice(alphabet) for _ in range(n))


def _hashes(seq, params, d=2, g=0, **kw):
    from ccj_amd import W_final
    wf = W_final(seq, d, params=params, noGU=bool(g), **kw)
    try:
        wf.fill()
        try:
            wf.result()
        except Exception:
            pass  # reference backtrack exits; the matrices are complete
        return wf.hashes()
    finally:
        wf.close()


CASES = [c for c in golden("hashes.json") if len(c["seq"]) >= 12][::3]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{len(c['seq'])}-{c['params']}-d{c['dangles']}-g{c['noGU']}")
def test_sharing_on_every_level_matches_reference(case):
    got = _hashes(case["seq"], case["params"], case["dangles"], case["noGU"], split_target=-1)
    bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
    assert not bad, f"matrices differ from the reference: {bad}"


@pytest.mark.parametrize("seed", range(6))
def test_sharing_random_inputs_match_oracle(seed):
    r = random.Random(3100 + seed)
    n = r.randint(30, 70)
    seq = _rseq(4100 + seed, n, r.choice(["ACGU", "GGCCAU", "GCAU"]))
    params = r.choice(["Turner04", "DirksPierce09", "DirksPierce03", "CaoChen09"])
    o = OracleFold(seq, blob(params), 2, 0)
    try:
        assert _hashes(seq, params, split_target=-1) == o.hashes()
    finally:
        o.close()


@pytest.mark.parametrize("n,seed", [(90, 1), (140, 2)])
def test_sharing_on_off_identical(n, seed):
    """Default schedule (sharing on the unsplit levels) == sharing off == sharing everywhere."""
    seq = _rseq(seed, n)
    h_on = _hashes(seq, "Turner04")
    assert _hashes(seq, "Turner04", share_splits=-1) == h_on
    assert _hashes(seq, "Turner04", split_target=-1) == h_on


def test_sharing_n400_same_result():
    """BASELINE config-5 size (n = 400, past the stock reference's n >= 214 abort): sharing on and
    off give the same MFE, structure and W array (full hashes would copy 47 GB to the host)."""
    from ccj_amd import W_final
    n = 400
    seq = _rseq(6, n)
    out = []
    for kw in ({}, {"share_splits": -1}):
        wf = W_final(seq, 2, params="Turner04", **kw)
        try:
            e = wf.ccj()
            out.append((e, wf.structure, [wf.W(j) for j in range(n + 1)]))
        finally:
            wf.close()
    assert out[0] == out[1]
    assert len(out[0][1]) == n and out[0][0] == out[0][2][n] / 100.0
