"""CPU tests: the C restatement of the fill (oracle/ccj_oracle.c) against fixtures produced by
the real reference (oracle/gen_golden.py -> tests/golden/hashes.json).  Every DP matrix must
hash identically (bit-exact int16/int32 contents in canonical (i,j,k,l) order)."""
import os

import pytest

from tests.oracle_lib import OracleFold, blob, golden

CASES = golden("hashes.json")
SMALL = CASES


@pytest.mark.parametrize("case", SMALL, ids=lambda c: f"n{len(c['seq'])}-{c['params']}-d{c['dangles']}-g{c['noGU']}")
def test_oracle_matches_reference(case):
    o = OracleFold(case["seq"], blob(case["params"]), case["dangles"], case["noGU"])
    try:
        got = o.hashes()
        bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
        assert not bad, f"matrices differ from reference: {bad}"
        assert o.W(len(case["seq"])) == case["mfe"]
    finally:
        o.close()


def test_golden_coverage():
    """The fixtures cover every parameter set, dangle model, noGU, and edge sizes."""
    e2e = golden("e2e.json")
    assert {c["params"] for c in e2e} >= {"Turner04", "DirksPierce09", "DirksPierce03", "CaoChen06", "CaoChen09",
                                          "DNA_Mathews2004"}
    assert {c["dangles"] for c in e2e} == {0, 1, 2}
    assert any(c["noGU"] for c in e2e)
    assert min(len(c["seq"]) for c in e2e) == 1
    assert any(c["rc"] != 0 for c in e2e), "an error path of the reference backtrack is covered"
    # the reference's "Should not be here!" side channel (W_final.cc:715) appears only at the
    # BASELINE sizes (rand100 seed 3, rand200 seed 5): those goldens must carry it
    assert any("Should not be here!" in c["stdout"] for c in golden("e2e_large.json"))
    trna = [c for c in e2e if c["seq"] == "GCGGAUUUAGCUCAGUUGGGAGAGCGCCAGAC" and c["params"] == "Turner04"
            and c["dangles"] == 2 and not c["noGU"]]
    assert trna and trna[0]["stdout"].splitlines()[-1] == ".........((((..[[[[..)))).]]]].. (-8.54)"


@pytest.mark.parametrize("case", CASES[::7], ids=lambda c: f"n{len(c['seq'])}-{c['params']}-d{c['dangles']}-g{c['noGU']}")
def test_level_parallel_oracle_matches_reference(case):
    """The level-parallel restatement (ccj_oracle_fold_par: spans and levels in the wavefront order
    of SURVEY.md F4, OpenMP threads) reproduces the reference's matrices exactly."""
    o = OracleFold(case["seq"], blob(case["params"]), case["dangles"], case["noGU"], threads=4)
    try:
        got = o.hashes()
        bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
        assert not bad, f"matrices differ from reference: {bad}"
        assert o.W(len(case["seq"])) == case["mfe"]
    finally:
        o.close()


def test_level_parallel_oracle_matches_reference_n100():
    """n=100 (BASELINE config 2's sequence): the parallel restatement against the reference's 31 hashes."""
    case = [c for c in golden("hashes_large.json") if c["tag"] == "t04_100"][0]
    o = OracleFold(case["seq"], blob(case["params"]), 2, 0, threads=0)
    try:
        got = o.hashes()
        assert got == case["hashes"]
        assert o.W(100) == case["mfe"]
    finally:
        o.close()


def test_level_parallel_oracle_matches_reference_n200():
    """n=200 (the headline bench sequence, t04_200) in the default CPU suite: the level-parallel
    restatement the config-5 fixtures (hashes_n400.json) rest on, against the reference's 31 hashes."""
    case = [c for c in golden("hashes_large.json") if c["tag"] == "t04_200"][0]
    o = OracleFold(case["seq"], blob(case["params"]), 2, 0, threads=int(os.environ.get("CCJ_ORACLE_THREADS", "0")))
    try:
        got = o.hashes()
        assert got == case["hashes"]
        assert o.W(200) == case["mfe"]
    finally:
        o.close()


SLOW = os.environ.get("CCJ_SLOW_TESTS") == "1"


@pytest.mark.skipif(not SLOW, reason="minutes per case on 8 cores: run with CCJ_SLOW_TESTS=1 "
                    "(log of the last run: profiles/r4_oracle_par_large.log)")
@pytest.mark.parametrize("tag", ["t04_150", "dp09_200", "t04_220", "dp09_230"])
def test_level_parallel_oracle_matches_reference_large(tag):
    """The level-parallel restatement against the reference's 31 matrix hashes at the BASELINE
    sizes and past the stock abort (n=220 / 230: the reference's own sources built with -DNDEBUG,
    matrices.hh:159-160).  This is what the n=400 fixture (hashes_n400.json) rests on."""
    case = [c for c in golden("hashes_large.json") if c["tag"] == tag][0]
    n = len(case["seq"])
    o = OracleFold(case["seq"], blob(case["params"]), case["dangles"], case["noGU"],
                   threads=int(os.environ.get("CCJ_ORACLE_THREADS", "0")))
    try:
        got = o.hashes()
        bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
        assert not bad, f"matrices differ from reference: {bad}"
        assert o.W(n) == case["mfe"]
    finally:
        o.close()
