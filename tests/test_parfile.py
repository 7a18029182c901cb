"""CPU tests of the native .par reader (include/ccj_parfile.h, ccj_amd/csrc/ccj_params_io.cc).

Pinned by
  * tests/golden/par_cases.json — synthetic .par texts run through the REAL reference loader
    (oracle/gen_par_golden.py: oracle/_ref/ref_driver dump-params), covering comments, '*',
    'x', DEF/INF/NST, shifted slices, update_nst, special-hairpin quirks, symmetry warnings,
    unknown identifiers and every fatal error — expected tables, stderr and exit status;
  * the bundled blobs ccj_amd/params/*.ccjp (ref_driver dumps of the reference's own parameter
    files): when /root/reference/params is present the files themselves are parsed and must give
    the same bytes (skipped elsewhere; the reference never travels).
"""
import base64
import ctypes
import hashlib
import os
import zlib

import pytest

from tests.oracle_lib import ROOT, golden

import ccj_amd
from ccj_amd import ParFileError, load_par

PARAMS = os.path.join(ROOT, "ccj_amd", "params")
REF_PARAMS = "/root/reference/params"
SETS = {"rna_Turner04": "Turner04", "rna_DirksPierce09": "DirksPierce09", "rna_DirksPierce03": "DirksPierce03",
        "rna_CaoChen06": "CaoChen06", "rna_CaoChen09": "CaoChen09", "dna_Matthews04": "Matthews04"}

# field layout of ccj_energy_params (include/ccj_params.h) for readable mismatch reports
_FIELDS = [("header", 16), ("stack", 4 * 64), ("hairpin", 4 * 31), ("bulge", 4 * 31), ("internal_loop", 4 * 31)]
_FIELDS += [(n, 4 * 200) for n in ("mismatchExt", "mismatchI", "mismatch1nI", "mismatch23I", "mismatchH", "mismatchM")]
_FIELDS += [("dangle5", 4 * 40), ("dangle3", 4 * 40), ("int11", 4 * 1600), ("int21", 4 * 8000),
            ("int22", 4 * 40000), ("scalars", 4 * 5), ("MLintern", 32), ("pad", 8), ("lxc", 8),
            ("Tetraloop_E", 800), ("Triloop_E", 160), ("Hexaloop_E", 160), ("Tetraloops", 1408),
            ("Triloops", 248), ("Hexaloops", 1808)]


def _field(off):
    for name, size in _FIELDS:
        if off < size:
            return f"{name}+{off}"
        off -= size
    return f"?+{off}"


def _unpack(z):
    return zlib.decompress(base64.b64decode(z))


def _base():
    return open(os.path.join(PARAMS, "default.ccjp"), "rb").read()


def test_field_table_covers_blob():
    assert sum(s for _, s in _FIELDS) == len(_base())


CASES = golden("par_cases.json")["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_par_case_matches_reference(case, tmp_path):
    text = _unpack(case["text_z"])
    par = tmp_path / "case.par"
    par.write_bytes(text)
    base = _base()
    if case["rc"] != 0:
        with pytest.raises(ParFileError) as ei:
            load_par(str(par), base)
        assert ei.value.log == case["stderr"]
        return
    applied, blob, log = load_par(str(par), base)
    assert applied == 1
    if "stderr" in case:
        assert log == case["stderr"]
    else:
        assert log.count("\n") == case["stderr_lines"]
        assert hashlib.sha256(log.encode()).hexdigest() == case["stderr_sha256"]
    want = bytes(x ^ y for x, y in zip(base, _unpack(case["xor_z"])))
    if blob != want:
        bad = sorted({_field(i).split("+")[0] for i in range(len(blob)) if blob[i] != want[i]})
        pytest.fail(f"tables differ in {bad}")
    assert hashlib.sha256(blob).hexdigest() == case["blob_sha256"]


def test_string_loader_matches_file_loader_without_blank_lines(tmp_path):
    """vrna_params_load_from_string drops empty lines; on texts without them both readers agree."""
    base = _base()
    n = 0
    for case in CASES:
        text = _unpack(case["text_z"]).decode()
        if case["rc"] != 0 or "\n\n" in text or "\r" in text:
            continue
        par = tmp_path / (case["name"] + ".par")
        par.write_text(text)
        a = load_par(str(par), base)
        b = load_par(text, base, text=True)
        assert a == b, case["name"]
        n += 1
    assert n >= 4


def test_string_loader_drops_blank_lines(tmp_path):
    """A blank line ends a special-hairpin list in a file (and still appends a space) but
    vanishes from a string (strtok), so the list continues there."""
    base = _base()
    text = "## RNAfold parameter file v2.0\n# Triloops\nCAACG 680 2370\n\nGUUAC 690 1080\n"
    par = tmp_path / "tri.par"
    par.write_text(text)
    off = sum(s for n, s in _FIELDS[: [n for n, _ in _FIELDS].index("Triloops")])
    _, blob_s, _ = load_par(text, base, text=True)
    _, blob_f, _ = load_par(str(par), base)
    assert blob_s[off:off + 13] == b"CAACG GUUAC \x00"
    assert blob_f[off:off + 8] == b"CAACG  \x00"


def test_unreadable_and_empty_files(tmp_path):
    base = _base()
    applied, blob, log = load_par(str(tmp_path / "missing.par"), base)
    assert (applied, blob) == (0, base)
    assert log == f"WARNING: read_parameter_file():Can't open file {tmp_path / 'missing.par'}\n\n"
    empty = tmp_path / "empty.par"
    empty.write_text("")
    assert load_par(str(empty), base) == (0, base, "")


def test_bad_base_rejected():
    with pytest.raises(ccj_amd.CCJError):
        load_par("## RNAfold parameter file v2.0\n", b"\0" * len(_base()), text=True)


@pytest.mark.skipif(not os.path.isdir(REF_PARAMS), reason="reference parameter files not present")
@pytest.mark.parametrize("stem", sorted(SETS))
def test_reference_parameter_files_give_bundled_blobs(stem):
    applied, blob, log = load_par(os.path.join(REF_PARAMS, stem + ".par"))
    assert applied == 1
    assert blob == open(os.path.join(PARAMS, SETS[stem] + ".ccjp"), "rb").read()
    # dna_Matthews04.par has an asymmetric stack_enthalpies table: 4 warnings, like the reference
    assert log == ("WARNING: stacking enthalpies not symmetric\n" * 4 if stem == "dna_Matthews04" else "")


@pytest.mark.skipif(not os.path.isdir(REF_PARAMS), reason="reference parameter files not present")
def test_load_params_reads_par_files_natively():
    p = os.path.join(REF_PARAMS, "rna_Turner04.par")
    assert ccj_amd.load_params(p) == open(os.path.join(PARAMS, "Turner04.ccjp"), "rb").read()
