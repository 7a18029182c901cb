"""Band-sharded fills on the GPU (-m gpu): every shard's launches (partitioned k_level4d / k_iloop,
k_copies after the level exchange) run in one context (shard_simulate), so a fold split G ways
must reproduce the unsharded fold bit for bit — matrices against the reference's hashes, and
MFE/structure against the unsharded engine at BASELINE sizes.  (The exchange itself is one
in-place RCCL all-gather per matrix and level; its layout is tested with gloo in test_shard.py.)
"""
import random

import pytest

from tests.oracle_lib import golden

pytestmark = pytest.mark.gpu

HASHES = [c for c in golden("hashes.json") if len(c["seq"]) >= 40][:4]


def _rseq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("case", HASHES, ids=lambda c: f"n{len(c['seq'])}-{c['params']}")
def test_sharded_matrices_identical_to_reference(case, world):
    from ccj_amd import W_final
    wf = W_final(case["seq"], case["dangles"], params=case["params"], noGU=bool(case["noGU"]),
                 shard_world=world, shard_simulate=True)
    try:
        wf.fill()
        try:
            wf.result()
        except Exception:
            pass
        got = wf.hashes()
        bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
        assert not bad, f"sharded x{world}: matrices differ from the reference: {bad}"
    finally:
        wf.close()


@pytest.mark.parametrize("n,world", [(100, 2), (100, 5), (200, 4), (200, 8)])
def test_sharded_fold_equals_unsharded(n, world):
    from ccj_amd import W_final
    seq = _rseq(5 if n == 200 else 3, n)
    ref = W_final(seq, 2, params="Turner04")
    try:
        e0 = ref.ccj()
        h0 = ref.hashes()
        s0 = ref.structure
    finally:
        ref.close()
    wf = W_final(seq, 2, params="Turner04", shard_world=world, shard_simulate=True)
    try:
        e1 = wf.ccj()
        assert (e1, wf.structure) == (e0, s0)
        assert wf.hashes() == h0
    finally:
        wf.close()


@pytest.mark.parametrize("world", [4])
@pytest.mark.parametrize("case", [c for c in golden("e2e_large.json") if c["n"] == 200], ids=lambda c: c["tag"])
def test_sharded_fold_matches_reference_stdout(case, world):
    """BASELINE config 4 (DirksPierce09, n=200, 4 GPUs) and the headline sequence, band-sharded
    (shard_simulate), against the reference's own output for the same input."""
    from ccj_amd import W_final
    wf = W_final(case["seq"], case["dangles"], params=case["params"], shard_world=world, shard_simulate=True)
    try:
        e = wf.ccj()
        assert wf.stdout_msgs + case["seq"] + "\n" + f"{wf.structure} ({e:g})\n" == case["stdout"]
    finally:
        wf.close()
