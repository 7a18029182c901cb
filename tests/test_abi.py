"""CPU tests of the boundary and host logic: the C-ABI library loads and exports every symbol
include/*.h declares (no compute without a GPU), the work model, the level layout arithmetic,
the parameter blobs and the CLI's argument handling."""
import ctypes
import os
import random
import re

import pytest

from tests.oracle_lib import ROOT

LIB = os.path.join(ROOT, "ccj_amd", "lib", "libccj_hip.so")


def declared_symbols():
    names = set()
    for h in ("ccj.h", "ccj_parfile.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"\b(ccj_[a-z0-9_]+)\s*\(", txt):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    L = ctypes.CDLL(LIB)
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing


def test_num_cells():
    L = ctypes.CDLL(LIB)
    L.ccj_num_cells.restype = ctypes.c_uint64
    L.ccj_num_cells.argtypes = [ctypes.c_int]
    for n, c in [(32, 40920), (100, 4082925), (200, 65998350), (400, 1061326700)]:
        assert L.ccj_num_cells(n) == c


def test_work_model_matches_survey_scale():
    """R4/B at n=100/200 (SURVEY.md §8d quotes B = 6.29 GB / 205.4 GB from its own counter)."""
    L = ctypes.CDLL(LIB)
    L.ccj_work_model_seq.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    r = random.Random(3)
    s = "".join(r.choice("ACGU") for _ in range(100))
    out = (ctypes.c_double * 4)()
    assert L.ccj_work_model_seq(s.encode(), 0, out) == 0
    assert out[3] == 4082925
    total = out[0] + out[1]
    assert 0.9 * 6.29e9 < total < 1.05 * 6.29e9


REC_ONLY = (5, 6, 8, 9, 10, 12, 13, 16, 18, 19, 21)  # the record-carried matrices (ccj_engine.h REC_MASK)


def _mslot(x):
    """ccj_engine.h mslot: the 11 stored matrices in enum order, then the 11 record-carried ones."""
    below = sum(x > r for r in REC_ONLY)
    return 11 + below if x in REC_ONLY else x - below


def _layout(n, nm4=22):
    """Python restatement of the level-major layout (ccj_engine.h) — brute-force bijection check;
    nm4 = 11 (d4 without the record-carried matrices) or 22 (mat5, and the host mirror)."""
    off, lv = 0, {}
    for t in range(n):
        m = n - t - 2
        M = m * (m + 1) // 2 if m > 0 else 0
        lv[t] = (off, (t + 1) * M, M, m)
        off += nm4 * (t + 1) * M
    return lv, off


@pytest.mark.parametrize("n", [5, 9, 17, 24])
@pytest.mark.parametrize("nm4", [11, 22])
def test_level_layout_is_a_bijection(n, nm4):
    lv, total = _layout(n, nm4)
    assert sorted(_mslot(x) for x in range(22)) == list(range(22))
    seen = set()
    for x in range(22):
        if _mslot(x) >= nm4:
            continue
        for i in range(1, n + 1):
            for j in range(i, n + 1):
                for k in range(j + 2, n + 1):
                    for l in range(k, n + 1):
                        a, g, b = j - i, k - j, l - k
                        t, h = a + b, g - 2
                        base, C, M, m = lv[t]
                        s = _mslot(x)
                        e = base + s * C + a * M + h * m - h * (h - 1) // 2 + i - 1
                        assert base + s * C <= e < base + (s + 1) * C
                        seen.add(e)
    assert len(seen) == total


def test_param_blobs():
    from ccj_amd import load_params, PARAM_SETS
    import struct
    for name in set(PARAM_SETS.values()):
        b = load_params(name.replace(".ccjp", ""))
        magic, ver, size = struct.unpack_from("<III", b, 0)
        assert magic == 0x504A4343 and ver == 1 and size == len(b)


def test_cli_validation_paths(capsys):
    """CCJ.cc:23-36 messages and exit codes, no GPU needed (they fail before the fold)."""
    import io
    from ccj_amd.cli import run
    out, err = io.StringIO(), io.StringIO()
    assert run(["ACGUX"], stdout=out, stderr=err) == 1
    assert out.getvalue() == "Sequence contains character X that is not G,C,A,U, or T.\n"
    out = io.StringIO()
    assert run(["-i", "whatever.txt"], stdout=out, stderr=err) == 1
    assert out.getvalue() == "sequence is missing\n"
    out, err = io.StringIO(), io.StringIO()
    assert run(["-P", "/nonexistent.par", "ACGU"], stdout=out, stderr=err) == 1
    assert err.getvalue() == "Not a valid parameter file!\n"
    out = io.StringIO()
    assert run([], stdin=io.StringIO("\n"), stdout=out, stderr=err) == 1
    assert out.getvalue() == "sequence is missing\n"


def test_pf_footprint_counts_the_large_allocations():
    """ccj_pf_footprint (the basis of ccj_pf_create's up-front size check): at least
    the int32 4-D store, its copies, the split-loop records (22 ints per cell) and the two double
    window tables; host = the window tables."""
    import ctypes
    L = ctypes.CDLL(LIB)
    L.ccj_pf_footprint.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]
    L.ccj_pf_footprint.restype = None
    for n in (10, 100, 200):
        dev, host = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        L.ccj_pf_footprint(n, ctypes.byref(dev), ctypes.byref(host))
        cells = sum((t + 1) * (n - t - 2) * (n - t - 1) // 2 for t in range(n - 2))
        ie = 2 * (29 * 29 * (n + 1) * (n + 2) + 8) * 8  # + the compacted rows' 8-double tail pad
        assert host.value == ie
        assert dev.value >= ie + (21 + 2 + 22) * cells * 4
        assert dev.value <= 1.3 * (ie + (21 + 2 + 22) * cells * 4) + (64 << 20)


def _pf_items_upper(n):
    """k_pf_iloop work items of ccj_pf_create's enumeration (ccj_pf.cc, ccj_items.h item_row) when every
    pair can pair: one item per 64-lane chunk of each PL / PR / PM row."""
    tot = 0
    for t in range(n - 2):
        m = n - t - 2
        tot += max(0, t - 5) * sum((m - i) // 64 + 1 for i in range(1, m + 1))   # PL: a in [6, t]
        tot += max(0, t - 5) * sum(q // 64 + 1 for q in range(m))                # PR: a in [0, t-6]
        for h in range(m):                                                        # PM
            for j in range(1, n - h - 1):
                k = j + h + 2
                lo, hi = max(2, t - (n - k)), min(t - 2, j - 1)
                if lo <= hi:
                    tot += (hi - lo) // 64 + 1
    return tot


def test_pf_footprint_bounds_the_work_items():
    """rows longer than 64 cells (n=200) hold several items; the footprint must cover the
    items' exact upper bound on top of the 4-D store, its copies and the window tables."""
    import ctypes
    L = ctypes.CDLL(LIB)
    L.ccj_pf_footprint.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]
    L.ccj_pf_footprint.restype = None
    n = 200
    dev, host = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    L.ccj_pf_footprint(n, ctypes.byref(dev), ctypes.byref(host))
    cells = sum((t + 1) * (n - t - 2) * (n - t - 1) // 2 for t in range(n - 2))
    pmx = sum((n - t - 2) * n * (t + 1) for t in range(n - 2))
    items = _pf_items_upper(n)
    assert dev.value >= host.value + (21 + 2) * cells * 4 + pmx * 4 + items * 4
