"""Partition function on the GPU against the reference's own W_final_pf.

tests/golden/pf_golden.json holds, per case, what src/part_func.cc (-ffp-contract=off) produced:
the ensemble energy, the IEEE bits of W[0..n], FNV-1a hashes of the 8 2-D matrices (IEEE bits)
and of the 21 4-D matrices (their int32 values, canonical order), and for some cases 5 stochastic
samples after srand(seed) — or the reference's "backtracking failed" line where it exits.
The bar is bit-identity: the fill evaluates every sum in the reference's order without
contraction.
"""
import json
import math
import os

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pf_golden.json")

with open(GOLD) as _f:
    CASES = json.load(_f)["cases"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_pf_matches_reference(case):
    import struct

    import ccj_amd
    pf = ccj_amd.W_final_pf(case["seq"], dangle=case["dangles"], params=case["params"])
    try:
        e = pf.ccj_pf()
        assert repr(e) == repr(float(case["energy"])) or (e != e and case["energy"] == "nan")
        wbits = ["%016x" % struct.unpack("<Q", struct.pack("<d", w))[0] for w in pf.W()]
        assert wbits == case["wbits"]
        h = pf.hashes()
        bad = {k: (h[k], v) for k, v in {**case["h2"], **case["h4"]}.items() if h[k] != v}
        assert not bad
        assert pf.exp_hashes() == case["exp"]
        if "srand" in case:
            pf.srand(case["srand"])
            try:
                got = pf.sample(5)
                assert "sample_exit" not in case
                assert got == case["samples"]
            except ccj_amd.SampleExit as ex:
                assert ex.structures == case["samples"]
                assert ex.stdout == case["sample_exit"]
    finally:
        pf.close()


@pytest.mark.gpu
def test_pf_refill_is_identical():
    import ccj_amd
    c = next(c for c in CASES if c["name"] == "big40_default")
    pf = ccj_amd.W_final_pf(c["seq"], params=c["params"])
    try:
        e1, h1 = pf.ccj_pf(), pf.hashes()
        e2, h2 = pf.ccj_pf(), pf.hashes()
        assert repr(e1) == repr(e2) and h1 == h2
    finally:
        pf.close()


@pytest.mark.gpu
def test_pf_rejects_bad_input():
    import ccj_amd
    with pytest.raises(ccj_amd.CCJError):
        ccj_amd.W_final_pf("ACGX")
    with pytest.raises(ccj_amd.CCJError):
        ccj_amd.W_final_pf("A" * 1100)


@pytest.mark.gpu
def test_pf_past_295_checks_exactness():
    """n >= 296 is no longer refused up front: the fill sums every P exactly and reports
    CCJ_E_PF_RANGE (10) only where sum |terms| >= 2^53 could make the reference's serial double
    sum round differently; poly-A has no pairs, so every P is 0 and the fold completes."""
    import ccj_amd
    pf = ccj_amd.W_final_pf("A" * 300, params="DirksPierce09")
    try:
        e = pf.ccj_pf()
        # Z = W[n] = 1 and pf_scale = 1: -log(1) * kT / 1000 = -0.0, as the reference prints for
        # poly-A ("ENERGY -0", oracle/_ref/pf_driver on A*30)
        assert e == 0.0 and math.copysign(1.0, e) == -1.0
        assert all(v == 1.0 for v in pf.W())
    finally:
        pf.close()


@pytest.mark.gpu
def test_pf_size_check_boundary(monkeypatch):
    """ccj_pf_create's up-front size check: with the device's free memory set to exactly the bytes
    ccj_pf_footprint reports (CCJ_PF_DEVMEM_LIMIT, a test hook) the context is created; one byte
    less fails with CCJ_E_OOM (2) before any table is built."""
    import ctypes
    import ccj_amd
    L = ccj_amd.lib()
    L.ccj_pf_footprint.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]
    L.ccj_pf_footprint.restype = None
    seq = "GGGAAACCCAGCUUCGGCUGGGAAACCC"
    dev, host = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    L.ccj_pf_footprint(len(seq), ctypes.byref(dev), ctypes.byref(host))
    monkeypatch.setenv("CCJ_PF_DEVMEM_LIMIT", str(dev.value - 1))
    with pytest.raises(ccj_amd.CCJError) as ei:
        ccj_amd.W_final_pf(seq)
    assert ei.value.code == 2, ei.value
    monkeypatch.setenv("CCJ_PF_DEVMEM_LIMIT", str(dev.value))
    pf = ccj_amd.W_final_pf(seq)
    try:
        pf.ccj_pf()
    finally:
        pf.close()


@pytest.mark.gpu
def test_pf_range_exit(monkeypatch):
    """The exactness guard itself: with the bound lowered from 2^53 to 2^10 (CCJ_PF_RANGE_LOG2, a
    test hook), a sequence whose P sums carry large terms fails with CCJ_E_PF_RANGE (10) naming the
    interval, instead of returning a result."""
    import ccj_amd
    c = next(c for c in CASES if c["name"] == "big60_default")
    monkeypatch.setenv("CCJ_PF_RANGE_LOG2", "10")
    pf = ccj_amd.W_final_pf(c["seq"], params=c["params"])
    try:
        with pytest.raises(ccj_amd.CCJError) as ei:
            pf.ccj_pf()
        assert ei.value.code == 10, ei.value  # CCJ_E_PF_RANGE
    finally:
        pf.close()
    monkeypatch.delenv("CCJ_PF_RANGE_LOG2")
    pf = ccj_amd.W_final_pf(c["seq"], params=c["params"])
    try:
        assert repr(pf.ccj_pf()) == repr(float(c["energy"]))
    finally:
        pf.close()


@pytest.mark.gpu
def test_pf_after_other_contexts():
    """Device memory handed back by an MFE context is not zero: no read may depend on fresh memory
    (the PM interior loop once read e_stP past its table for j == 1, k == n)."""
    import ccj_amd
    for name in ("tetra_DirksPierce09", "big40_default", "knot_default"):
        wf = ccj_amd.W_final("GCGGAUUUAGCUCAGUUGGGAGAGCGCCAGAC", 2, params="Turner04")
        wf.ccj()
        wf.close()
        c = next(c for c in CASES if c["name"] == name)
        pf = ccj_amd.W_final_pf(c["seq"], dangle=c["dangles"], params=c["params"])
        try:
            e = pf.ccj_pf()
            h = pf.hashes()
            assert repr(e) == repr(float(c["energy"]))
            assert not [k for k, v in {**c["h2"], **c["h4"]}.items() if h[k] != v]
            if name == "tetra_DirksPierce09":  # the reference's value (oracle/_ref/pf_driver --dump4)
                assert pf.get4("PM", 1, 1, 32, 32) == 1 and pf.get4("PK", 1, 2, 4, 32) == 2580
        finally:
            pf.close()


GOLD_LARGE = os.path.join(os.path.dirname(__file__), "golden", "pf_golden_large.json")
LARGE = json.load(open(GOLD_LARGE))["cases"] if os.path.exists(GOLD_LARGE) else []


@pytest.mark.gpu
@pytest.mark.skipif(not LARGE, reason="tests/golden/pf_golden_large.json not generated (oracle/gen_pf_golden.py --large)")
@pytest.mark.parametrize("case", LARGE, ids=[c["name"] for c in LARGE])
def test_pf_matches_reference_large(case):
    """bench.py --pf's own workload (n=200, seed 5, Turner04) and n=150 DirksPierce09 against the
    reference's part_func.cc: every bit of W, all 29 matrices, the samples."""
    test_pf_matches_reference(case)


@pytest.mark.gpu
def test_pf_kernel_timing_and_work_model():
    """ccj_pf_set_timing / ccj_pf_kernel_ms / ccj_pf_work_model: every family timed in a timed fill,
    nothing in an untimed one, and the timed fill's results unchanged."""
    import ccj_amd
    c = next(c for c in CASES if c["name"] == "big60_default")
    pf = ccj_amd.W_final_pf(c["seq"], params=c["params"])
    try:
        pf.set_timing(True)
        e = pf.ccj_pf()
        km = pf.kernel_ms()
        assert repr(e) == repr(float(c["energy"]))
        assert set(km) == set(pf.PF_KERNELS) and all(v > 0 for v in km.values())
        assert sum(km.values()) < 10 * pf.fill_ms()
        pf.set_timing(False)
        pf.ccj_pf()
        assert all(v == 0 for v in pf.kernel_ms().values())
        w = pf.work_model()
        # the level kernel reads at least its 21 stores' worth per cell; every family does work
        assert w["k_pf_level"] >= 84 * ccj_amd.num_cells(60) and all(v > 0 for v in w.values())
    finally:
        pf.close()


PF_FUZZ = int(os.environ.get("CCJ_PF_FUZZ", "0"))
PF_DRV = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "pf_driver")


@pytest.mark.gpu
@pytest.mark.skipif(PF_FUZZ <= 0 or not os.path.exists(PF_DRV),
                    reason="opt-in randomized campaign against the reference's own part_func.cc: CCJ_PF_FUZZ=<cases>")
@pytest.mark.parametrize("k", range(max(PF_FUZZ, 1)))
def test_pf_fuzz_against_reference_driver(k):
    """Opt-in randomized campaign (round 6): a random sequence (n 6-50, dangles 0/1/2, the reference's
    default parameters) through oracle/_ref/pf_driver (the reference's W_final_pf, built here from its
    own sources with -ffp-contract=off) and through the GPU: the energy, the IEEE bits of W and every
    matrix hash identical."""
    import random
    import struct
    import subprocess

    import ccj_amd
    r = random.Random(70000 + k)
    n = r.randint(6, 50)
    seq = "".join(r.choice(r.choice(["ACGU", "GGCCAU", "GCAU"])) for _ in range(n))
    d = r.choice([0, 1, 2])
    p = subprocess.run([PF_DRV, seq, "-d", str(d)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-400:]
    ref = {"h2": {}, "h4": {}}
    for line in p.stdout.splitlines():
        w = line.split()
        if w and w[0] == "ENERGY":
            ref["energy"] = w[1]
        elif w and w[0] == "WBITS":
            ref["wbits"] = w[1:]
        elif w and w[0] in ("H2", "H4"):
            ref[w[0].lower()][w[1]] = w[2]
    pf = ccj_amd.W_final_pf(seq, dangle=d, params="default")
    try:
        e = pf.ccj_pf()
        assert repr(e) == repr(float(ref["energy"])) or (e != e and ref["energy"] == "nan"), (seq, d)
        assert ["%016x" % struct.unpack("<Q", struct.pack("<d", w))[0] for w in pf.W()] == ref["wbits"], (seq, d)
        h = pf.hashes()
        assert not {k2: v for k2, v in {**ref["h2"], **ref["h4"]}.items() if h[k2] != v}, (seq, d)
    finally:
        pf.close()
