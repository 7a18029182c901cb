#!/usr/bin/env python3
"""oracle/gen_par_golden.py — TEST INFRASTRUCTURE: golden vectors for the native .par reader.

Builds synthetic "RNAfold parameter file v2.0" texts that exercise every rule of the
reference loader (src/ViennaRNA/params/io.c:454-1299 + params.c:399-555): comments, '*' skips,
'x' extrapolation, DEF/INF/NST, per-block fresh lines, shifted N-d slices, update_nst, the
special-hairpin list quirks, symmetry warnings, unknown identifiers and the fatal errors.
Each text is loaded by the REAL reference (oracle/_ref/ref_driver dump-params -P FILE, built by
oracle/Makefile from /root/reference) on top of its compiled-in defaults, and the result is
recorded as data in tests/golden/par_cases.json:

  {"name", "text_z", "rc", "stderr" | "stderr_sha256"+"stderr_lines",
   "blob_sha256", "xor_z"}
  text_z = base64(zlib(.par text)); xor_z = base64(zlib(blob XOR default.ccjp)), so a mismatch
  can be reported field by field.

The .par texts are our own synthetic inputs (none of the reference's files are copied); the
reference itself never leaves this container.
"""
import base64
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
DEFAULT = os.path.join(ROOT, "ccj_amd", "params", "default.ccjp")
OUT = os.path.join(ROOT, "tests", "golden", "par_cases.json")
HDR = "## RNAfold parameter file v2.0\n"


def rows(vals, per=8):
    return "".join(" ".join("%6s" % v for v in vals[i:i + per]) + "\n" for i in range(0, len(vals), per))


def sym_int22(rng, lo=-40, hi=90):
    """int22 values for pairs 1..6 x 1..6 and bases 1..4 that are symmetric under
    (i,j,k,l,m,n) -> (j,i,m,n,k,l), emitted in the reader's order (one 4-value block per (i,j,k,l,m))."""
    v = {}
    for i in range(1, 7):
        for j in range(1, 7):
            for k in range(1, 5):
                for l in range(1, 5):
                    for m in range(1, 5):
                        for n in range(1, 5):
                            key = (i, j, k, l, m, n)
                            mate = (j, i, m, n, k, l)
                            if mate in v:
                                v[key] = v[mate]
                            else:
                                v[key] = rng.randint(lo, hi)
    out = []
    for i in range(1, 7):
        for j in range(1, 7):
            for k in range(1, 5):
                for l in range(1, 5):
                    for m in range(1, 5):
                        out.append(" ".join("%5d" % v[(i, j, k, l, m, n)] for n in range(1, 5)))
    return v, "\n".join(out) + "\n"


def cases():
    rng = random.Random(2024)
    c = {}
    # 1 stack: comments, DEF/INF/NST, '*', one asymmetric pair (2 warnings)
    st = []
    for i in range(1, 8):
        st.append(" ".join("%5d" % (-100 * min(i, j) - 10 * max(i, j)) for j in range(1, 8)))
    st[2] = "/* row with a comment */ " + st[2]
    st[3] = st[3].split()
    st[3][0], st[3][5], st[3][6] = "DEF", "*", "INF"
    st[3] = " ".join(st[3]) + "   /* trailing */"
    st[4] = st[4].replace(st[4].split()[1], "NST", 1)
    c["stack_tokens"] = HDR + "\n# stack\n" + "\n".join(st) + "\n\n#END\n"
    # 2 no header; hairpin with x extrapolation, extra tokens dropped, bulge/interior
    hp = ["INF", "INF", "INF", "540", "560", "570", "540", "600", "550", "640"] + ["x"] * 21
    c["no_header_extrap"] = ("# hairpin\n" + " ".join(hp[:12]) + "\n" + " ".join(hp[12:]) + " 999 999\n"
                             "# bulge\n" + " ".join(["INF", "380", "280", "320", "360", "400", "440"] + ["x"] * 24) +
                             "\n# interior\nINF INF INF INF 110 200 200 210 230 240 250\n" + " ".join(["x"] * 20) +
                             "\n")
    # 3 clamped tables: mismatch_multi / mismatch_exterior / dangles with positive entries
    mm = "".join(rows([rng.randint(-120, 60) for _ in range(25)], 5) for _ in range(7))
    dg = "".join("%5d %5d %5d %5d %5d\n" % tuple(rng.randint(-60, 40) for _ in range(5)) for _ in range(7))
    c["clamps"] = (HDR + "# mismatch_multi\n" + mm + "# mismatch_exterior\n" + mm.replace("-", " ") +
                   "# mismatch_hairpin\n" + mm + "# mismatch_interior_1n\n" + mm + "# dangle5\n" + dg +
                   "# dangle3\n" + dg.replace("-", "+") + "# dangle5_enthalpies\n" + dg + "#END\n")
    # 4 int11 with asymmetric entries + enthalpies, int21
    i11 = "".join(rows([rng.randint(-50, 200) for _ in range(25)], 5) for _ in range(49))
    i21 = "".join(rows([rng.randint(0, 90) for _ in range(125)], 5) for _ in range(49))
    c["int11_int21"] = (HDR + "# int11\n" + i11 + "# int11_enthalpies\n" + i11 + "# int21\n" + i21 +
                        "# int21_enthalpies\n" + i21 + "#END\n")
    # 5 int22 (symmetric) -> update_nst; enthalpies with one asymmetric entry
    v, txt = sym_int22(rng)
    lines = txt.splitlines()
    bad = lines[7].split()
    bad[3] = str(int(bad[3]) + 17)
    lines_h = list(lines)
    lines_h[7] = " ".join(bad)
    c["int22_nst"] = HDR + "# int22\n" + txt + "# int22_enthalpies\n" + "\n".join(lines_h) + "\n#END\n"
    # 6 special hairpins: short sequence gap, 2-field line ends the list, swallowed header
    c["loops_quirks"] = (HDR + "# Tetraloops\nCAACGG 550 690\nGAAA 300 200\nCCAAGG 330 -1030\n\n"
                         "# Triloops\nCAACG 680 2370\nGUUAC 690 1080\nAGAAU 700\n"
                         "# Hexaloops\nACAGUACU 280 -1680\nACAGUGAU 360 -1140\n# Tetraloops\n"
                         "GGGGAC -300 -100\n# Triloops\nCAACG 100 200\n\n#END\n")
    c["loops_full"] = (HDR + "# Tetraloops\n" + "".join("%s %d %d\n" % ("".join(rng.choice("ACGU") for _ in range(6)),
                                                                         rng.randint(-300, 600), rng.randint(-2000, 0))
                                                          for _ in range(40)) +
                       "UUUUUU 1 1\n# Hexaloops\n\n#END\n")
    # 7 scalars + duplicate section (later wins, '*' keeps the earlier value)
    c["scalars"] = (HDR + "# ML_params\n/* F = cu*n_unpaired + cc + ci*loop_degree */\n"
                    "\t    0\t    0\t  930\t 3000\t  -90\t -220\n"
                    "# NINIO\n/* Ninio = MIN(max, m*|n1-n2| */\n\t   60\t  320\t  300\n"
                    "# Misc\n/* all parameters are pairs of 'energy enthalpy' */\n   410  360    50   370\n"
                    "# stack\n" + rows(list(range(-49, 0)), 7) + "# stack\n" + rows(["*"] * 10 + list(range(100, 139)), 7) +
                    "#END\n")
    # 8 identifiers: unknown, '##' lines, bare '#', tokens split at 15 chars, 12abc, +5
    c["identifiers_tokens"] = (HDR + "# bogus_section\n1 2 3\n## RNAfold parameter file v2.0\n#\n"
                               "#    hairpin\nINF INF 123456789012345678 12abc +5 -7 " + " ".join(["300"] * 30) + "\n"
                               "#END\n# dangle3\n" + "".join("-1 -2 -3 -4 -5\n" for _ in range(7)))
    # 9 CRLF line endings
    c["crlf"] = (HDR + "# bulge\n" + " ".join(str(x) for x in range(31)) + "\n").replace("\n", "\r\n")
    # 10 fatal errors (reference: vrna_message_error + exit(1))
    c["fatal_bad_token"] = HDR + "# stack\n1 2 3 4 5 6 7\n1 2 abc 4 5 6 7 tail tokens\n"
    c["fatal_unclosed_comment"] = HDR + "# hairpin\nINF INF /* open comment\n"
    c["fatal_eof"] = HDR + "# hairpin\nINF INF 100\n"
    c["fatal_extrapolate_first"] = HDR + "# interior\nx 1 2\n"
    c["fatal_bare_sign"] = HDR + "# NINIO\n60 - 300\n"
    c["warn_then_fatal"] = "no header\n# what\n# bulge\n1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18 19 20 " \
                           "21 22 23 24 25 26 27 28 29 30 31\n# stack\n1 2 3\n#xyz\n"
    return c


def run_ref(text):
    with tempfile.TemporaryDirectory() as d:
        par = os.path.join(d, "case.par")
        blob = os.path.join(d, "case.ccjp")
        with open(par, "w", newline="") as f:
            f.write(text)
        r = subprocess.run([DRV, "dump-params", "-P", par, "-o", blob], capture_output=True, text=True, timeout=120)
        data = open(blob, "rb").read() if (r.returncode == 0 and os.path.exists(blob)) else None
    return r.returncode, r.stderr, data


def pack(b):
    return base64.b64encode(zlib.compress(b, 9)).decode()


def main():
    if not os.path.exists(DRV):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    base = open(DEFAULT, "rb").read()
    out = []
    for name, text in cases().items():
        rc, err, blob = run_ref(text)
        rec = {"name": name, "text_z": pack(text.encode()), "rc": rc}
        if len(err) <= 8192:
            rec["stderr"] = err
        else:
            rec["stderr_sha256"] = hashlib.sha256(err.encode()).hexdigest()
            rec["stderr_lines"] = err.count("\n")
        if blob is not None:
            rec["blob_sha256"] = hashlib.sha256(blob).hexdigest()
            rec["xor_z"] = pack(bytes(x ^ y for x, y in zip(base, blob)))
        out.append(rec)
        print(name, rc, len(err), len(rec.get("xor_z", "")))
    with open(OUT, "w") as f:
        json.dump({"generator": "oracle/gen_par_golden.py", "base": "ccj_amd/params/default.ccjp", "cases": out}, f,
                  indent=1)


if __name__ == "__main__":
    main()
