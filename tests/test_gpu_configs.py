"""One named parity test per BASELINE.json config (-m gpu), each against a fixture of the
reference or of the pinned restatement, through the product path (libccj_hip.so):

  config 1  32-nt tRNA fragment, Turner04: every DP matrix against the C oracle, stdout line
            against the reference CLI golden (tests/golden/e2e.json)
  config 2  100-nt random (seed 3), Turner04: 31 reference hashes + the reference's stdout
  config 3  200-nt headline (seed 5), Turner04: 31 reference hashes + the reference's stdout
            (the bench.py default sequence)
  config 4  200-nt DirksPierce09 (seed 5), 4 ranks band-sharded through the exchange path (in-process
            group: own blocks, pack, one all-gather per level, unpack), every rank against the
            reference's 31 hashes and stdout
  config 5  400-nt (seed 6, the first sequence of the 8-GPU batch), Turner04: 31 hashes + MFE against
            tests/golden/hashes_n400.json — restatement-pinned (oracle/ccj_oracle.c level-parallel
            mode, itself checked against every reference fixture up to n=230), not a reference run:
            the reference needs ~12 h per n=400 fold and its stock build aborts at n >= 214.
"""
import os

import pytest

from tests.oracle_lib import GOLDEN, golden

pytestmark = pytest.mark.gpu


def _large(tag):
    return [c for c in golden("hashes_large.json") if c["tag"] == tag][0]


def _fold_and_check(case, allow_exit=False, **kw):
    """Fold, require the fixture's 31 matrix hashes and W(n); return (structure, energy), or with
    allow_exit the reference's own backtrack exit as (None, BacktrackExit)."""
    from ccj_amd import W_final, BacktrackExit
    wf = W_final(case["seq"], case["dangles"], params=case["params"], noGU=bool(case["noGU"]), **kw)
    try:
        wf.fill()
        try:
            e = wf.result()
            out = (wf.structure, e)
        except BacktrackExit as ex:
            if not allow_exit:
                raise
            out = (None, ex)
        got = wf.hashes()
        bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
        assert not bad, f"matrices differ from the fixture: {bad}"
        assert wf.W(case["n"]) == case["mfe"]
        return out
    finally:
        wf.close()


def test_config1_trna32_turner04():
    from ccj_amd import W_final
    from tests.oracle_lib import OracleFold, blob
    seq = "GCGGAUUUAGCUCAGUUGGGAGAGCGCCAGAC"
    wf = W_final(seq, 2, params="Turner04")
    o = OracleFold(seq, blob("Turner04"), 2, 0)
    try:
        e = wf.ccj()
        assert wf.hashes() == o.hashes()
        ref = [c for c in golden("e2e.json") if c["seq"] == seq and c["params"] == "Turner04" and c["dangles"] == 2
               and not c["noGU"]][0]
        assert wf.stdout_msgs + seq + "\n" + f"{wf.structure} ({e:g})\n" == ref["stdout"]
    finally:
        wf.close()
        o.close()


def test_config2_random100_turner04():
    case = _large("t04_100")
    s, e = _fold_and_check(case)
    assert f"{s} ({e:g})" == case["stdout"].splitlines()[-1]


def test_config3_headline200_turner04():
    case = _large("t04_200")
    assert case["seed"] == 5 and case["n"] == 200  # bench.py's default sequence
    s, e = _fold_and_check(case)
    assert f"{s} ({e:g})" == case["stdout"].splitlines()[-1]


def test_config4_dp09_200_four_ranks_exchange():
    from tests.test_gpu_shard import _close_group, _fold_group
    case = _large("dp09_200")
    g, ranks = _fold_group(case["seq"], case["params"], 4)
    try:
        for wf in ranks:
            e = wf.result()
            assert f"{wf.structure} ({e:g})" == case["stdout"].splitlines()[-1]
            got = wf.hashes()
            assert {k: got[k] for k in case["hashes"]} == case["hashes"]
    finally:
        _close_group(g, ranks)


N400 = os.path.join(GOLDEN, "hashes_n400.json")


def _n400_seeds():
    return sorted(c["seed"] for c in golden("hashes_n400.json")) if os.path.exists(N400) else []


TB400 = os.path.join(GOLDEN, "traceback_n400.json")


def _tb400(seed):
    """The expected traceback outcome of an n=400 seed (oracle/gen_traceback_n400.py: the host restatement of
    the reference backtrack over matrices equal to the fixture), or None when not recorded yet."""
    if not os.path.exists(TB400):
        return None
    hit = [c for c in golden("traceback_n400.json") if c["seed"] == seed]
    return hit[0] if hit else None


@pytest.mark.skipif(not os.path.exists(N400), reason="tests/golden/hashes_n400.json not generated yet "
                                                     "(oracle/gen_hashes_n400.py)")
@pytest.mark.parametrize("seed", _n400_seeds())
def test_config5_batch400(seed):
    """Config 5's sequences (seeds 6.. of the 8-GPU batch): every seed the fixture holds.  The device
    traceback must give the recorded outcome: the structure and energy, or, only where the record says so,
    the reference's own impossible-case exit (pseudo_loop.cc:1081, P_PR), which the reference itself takes
    on some sequences (one of the 16 n=200 folds of profiles/r5_ref_allcores_n200.json).  A seed without a
    record must give a structure."""
    case = [c for c in golden("hashes_n400.json") if c["seed"] == seed][0]
    assert case["n"] == 400
    tb = _tb400(seed)
    expect_exit = tb is not None and "exit" in tb
    s, e = _fold_and_check(case, allow_exit=expect_exit)
    if expect_exit:
        assert s is None, f"expected the recorded exit, got a structure ({e})"
        assert e.exit_code == tb["exit"]["code"] and e.msg == tb["exit"]["msg"], e.msg
    else:
        assert round(e * 100) == case["mfe"] and len(s) == 400
        if tb is not None:
            assert s == tb["structure"] and e == tb["energy"]
