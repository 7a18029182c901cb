"""Full-matrix parity at BASELINE sizes and past the stock n >= 214 abort (-m gpu).

tests/golden/hashes_large.json holds, per case, the real reference's stdout (W_final::ccj) and an
FNV-1a hash of every DP matrix (22 four-dimensional, P/WBP/WPP/V/Vtype/WM/WMv/WMp, W) after its
fill (oracle/gen_hashes_large.py: oracle/_ref/ref_driver fold --hash, n=100..200 with the stock
build; n=220/230 with the same sources built -DNDEBUG, since the stock build asserts at
matrices.hh:160 for n >= 214 and is otherwise identical).  Each case is checked unsharded, and
band-sharded with every shard's launches in one context (shard_simulate) — world 4 is BASELINE
config 4 (DirksPierce09, n=200, 4 GPUs).
"""
import pytest

from tests.oracle_lib import golden

pytestmark = pytest.mark.gpu

CASES = golden("hashes_large.json")


def _check(case, **kw):
    from ccj_amd import W_final
    wf = W_final(case["seq"], case["dangles"], params=case["params"], noGU=bool(case["noGU"]), **kw)
    try:
        e = wf.ccj()
        got = wf.hashes()
        bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
        assert not bad, f"matrices differ from the reference: {bad}"
        assert wf.W(len(case["seq"])) == case["mfe"]
        assert f"{wf.structure} ({e:g})" == case["stdout"].splitlines()[-1]
    finally:
        wf.close()


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["tag"])
def test_large_matrices_identical_to_reference(case):
    _check(case)


@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("case", [c for c in CASES if c["n"] >= 200], ids=lambda c: c["tag"])
def test_large_sharded_matrices_identical_to_reference(case, world):
    _check(case, shard_world=world, shard_simulate=True)


@pytest.mark.parametrize("case", [c for c in CASES if c["n"] == 200], ids=lambda c: c["tag"])
def test_large_no_split_sharing_identical_to_reference(case):
    _check(case, share_splits=-1)
