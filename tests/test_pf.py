"""Partition function — host side, on CPU.

The golden vectors (tests/golden/pf_golden.json, oracle/gen_pf_golden.py) come from the
reference's own W_final_pf (src/part_func.cc + stoch_backtrack.cc) built with
-ffp-contract=off.  Here: the file is complete and self-consistent, and the Boltzmann tables this
package computes on the host (include/ccj_pf.h ccj_pf_exp_hashes_params: get_scaled_exp_params
+ rescale_pk_globals restated) are bit-identical to the reference's for every parameter set the
goldens use.  The GPU fill is checked against the same file in tests/test_gpu_pf.py.
"""
import json
import os
import struct

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pf_golden.json")


def _cases():
    with open(GOLD) as f:
        return json.load(f)["cases"]


def test_golden_file_complete():
    from ccj_amd import PF_MAT2, PF_MAT4
    cs = _cases()
    assert len(cs) >= 50
    names = set()
    for c in cs:
        assert c["name"] not in names
        names.add(c["name"])
        n = len(c["seq"])
        assert len(c["wbits"]) == n + 1
        assert sorted(c["h4"]) == sorted(PF_MAT4)
        assert sorted(c["h2"]) == sorted(PF_MAT2)
        # W[0..TURN] keep their initial scale[1] == 1.0 (part_func.cc:92)
        assert all(w == "3ff0000000000000" for w in c["wbits"][:min(n, 3) + 1])
        # the energy is to_Energy(W[n], n) = -log(W[n]) * kT / 1000 with pf_scale 1
        wn = struct.unpack("<d", bytes.fromhex(c["wbits"][n])[::-1])[0]
        if wn > 0:
            import math
            kT = 1.0 * (37.0 + 273.15) * 1.98717
            assert float(c["energy"]) == (-math.log(wn) - n * math.log(1.0)) * kT / 1000.0
    # both parameter sets, every dangles model, special hairpins, sampling incl. failure paths
    assert {c["params"] for c in cs} >= {"default", "DirksPierce09"}
    assert {c["dangles"] for c in cs} == {0, 1, 2}
    assert any("sample_exit" in c for c in cs)
    assert any(c.get("samples") for c in cs)


def _exp_sets():
    with open(GOLD) as f:
        return json.load(f)["exp_sets"]


@pytest.mark.parametrize("params", ["default", "Turner04", "DirksPierce09", "DirksPierce03", "CaoChen06", "CaoChen09",
                                    "Matthews04", "DNA_Mathews2004"])
def test_boltzmann_tables_match_reference(params):
    """Every bundled set, with its .pfraw raw tables, against scale_pf_parameters() of the reference."""
    import ccj_amd
    try:
        ccj_amd.lib()
    except ccj_amd.CCJError:
        pytest.skip("libccj_hip.so not built")
    ref = _exp_sets()[params]
    assert ccj_amd.pf_exp_hashes(params) == ref
    for c in _cases():  # and what each golden case's own run printed
        if c["params"] == params:
            assert c["exp"] == ref


def test_raw_tables_shipped_for_every_bundled_set():
    import ccj_amd
    for name in ccj_amd.PARAM_SETS:
        raw = ccj_amd.load_pfraw(name)
        assert raw is not None and len(raw) == 1928, name
        magic, size = struct.unpack("<II", raw[:8])
        assert magic == 0x52434343 and size == 1928
        # every shipped set has the reference's INF in the whole pair-type-0 row (the fallback rule)
        vals = struct.unpack("<480i", raw[8:])
        d5, d3, mM, mE = vals[:40], vals[40:80], vals[80:280], vals[280:480]
        assert all(v == 10000000 for v in d5[:5] + d3[:5] + mM[:25] + mE[:25]), name


def test_row0_fallback_equals_raw_for_turner():
    """Without raw tables the type-0 rows are taken as INF: exact for the Turner 2004 sets."""
    import ccj_amd
    try:
        L = ccj_amd.lib()
    except ccj_amd.CCJError:
        pytest.skip("libccj_hip.so not built")
    import ctypes
    names = L.ccj_pf_exp_names().decode().split()
    blob = ccj_amd.load_params("default")
    out = (ctypes.c_uint64 * len(names))()
    assert L.ccj_pf_exp_hashes_params(bytes(blob), None, None, out, len(names)) == len(names)
    assert {k: "%016x" % v for k, v in zip(names, out)} == ccj_amd.pf_exp_hashes("default")
