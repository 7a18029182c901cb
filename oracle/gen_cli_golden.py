#!/usr/bin/env python3
"""oracle/gen_cli_golden.py — TEST INFRASTRUCTURE: golden vectors for the CCJ command line.

Runs the REAL reference CLI (oracle/_ref/CCJ, built by oracle/Makefile from /root/reference
src/CCJ.cc + src/cmdline.cc) with argv[0] = "CCJ" on a list of argument vectors / stdin texts /
extra files, in a scratch directory that holds params/rna_DirksPierce09.par (the default the
reference loads relative to its CWD), and records stdout, stderr and the exit status in
tests/golden/cli.json.  "fold" marks cases that reach the MFE fill (GPU tests); the others end
in the option parser, the sequence check or the parameter loader (CPU tests).
The extra files are our own synthetic .par texts; nothing of the reference is copied.
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "CCJ")
OUT = os.path.join(ROOT, "tests", "golden", "cli.json")
HDR = "## RNAfold parameter file v2.0\n"

BAD_PAR = HDR + "# stack\n1 2 3 4 5 6 7\n1 2 abc 4 5 6 7 tail\n"
WARN_PAR = "# what\n# ML_params\n0 0 500 3000 -50 -220\n# NINIO\n40 320 200\n# Misc\n0 0 80 370\n#END\n"
LOOP_PAR = (HDR + "# Tetraloops\nGGGGAC -1500 -100\nGAAA 300 200\n# Triloops\nGGAAC 50 10\n"
            "# Hexaloops\nACAGUACU -900 -1680\n\n#END\n")

S1 = "GGGGAAACCCC"
S2 = "GCGGAUUUAGCUCAGUUGGGAGAGCGCCAGAC"
S3 = "GGGCGCAAGCCUAAGGGCGCCCAUCCGAGGGCGCUUUU"


def cases():
    c = []

    def add(argv, stdin="", files=None, fold=False):
        c.append({"argv": argv, "stdin": stdin, "files": files or {}, "fold": fold})

    for a in (["--help"], ["-h"], ["-V"], ["--version"], ["--he"], ["--ver"], ["-h", "-V"], ["-V", "-h"], ["-hV"],
              ["ACGU", "--help"], ["-d", "abc", "-h"]):
        add(a)
    for a in (["--bogus"], ["--bogus=1"], ["-x"], ["-x", "-d"], ["-d"], ["--dangles"], ["--dang"], ["-i"],
              ["--input-file"], ["-P"], ["-d", "abc", "ACGU"], ["-d", "1x", "ACGU"], ["-dV"], ["-d", "", "ACGU"],
              ["-d", "-", "ACGU"], ["-d", " ", "ACGU"], ["-d", "08", "ACGU"], ["-d", "0x", "ACGU"],
              ["-d", "1", "-d", "2", "ACGU"], ["-d3", "-d", "2"], ["--noConv", "--noConv", "ACGU"],
              ["--noGU", "--noGU"], ["--no", "--noConv"], ["-i", "a", "-i", "b"], ["-P", "x", "-P", "y", "ACGU"],
              ["--noConv=1"], ["--noC=1", "ACGU"], ["--n=1"], ["--=x"], ["--="], ["--device", "1", "ACGU"],
              ["-D"], ["--paramfile", "x"]):
        add(a)
    add(["-i", "seq.txt"], stdin=S1 + "\n")
    add([], stdin="")
    add([], stdin="ACGX\n")
    add(["acgn"])
    add(["--", "-x"])
    add(["-", "ACGU"])
    add(["ACG U"])
    add(["--noConv", "ACGTX"])
    add(["-P", "nonexistent.par", "ACGU"])
    add(["--paramFile=", "ACGU"])
    add(["-P", "bad.par", "ACGU"], files={"bad.par": BAD_PAR})
    add(["-P", "bad.par", "ACGX"], files={"bad.par": BAD_PAR})
    add(["-P", "warn_bad.par", "ACGU"], files={"warn_bad.par": "# zzz\n" + BAD_PAR})
    # reach the fold (GPU)
    add([S1], fold=True)
    add([], stdin=S2.lower() + "\n", fold=True)
    add(["-d", "0", S2], fold=True)
    add(["-d", "0x1", S2], fold=True)
    add(["--dangles= 1", S3], fold=True)
    add(["--noGU", S3], fold=True)
    add(["--no", "GGGGAAAUCCCC"], fold=True)
    add(["GGGGAAAUCCCC", "--noConv"], fold=True)
    add(["--noConv", "GGGGAAATTCCCC"], fold=True)
    add(["ACGU", "extra", "args"], fold=True)
    add(["-P", "warn.par", S2], files={"warn.par": WARN_PAR}, fold=True)
    add(["-P", "loops.par", "GGGGGACCCCC" + "AAAAA" + "GGGAAACCC"], files={"loops.par": LOOP_PAR}, fold=True)
    add(["-P", "loops.par", "-d", "0", S3], files={"loops.par": LOOP_PAR}, fold=True)
    return c


def main():
    if not os.path.exists(REF):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    out = []
    for case in cases():
        with tempfile.TemporaryDirectory() as d:
            os.makedirs(os.path.join(d, "params"))
            shutil.copy("/root/reference/params/rna_DirksPierce09.par", os.path.join(d, "params"))
            for name, text in case["files"].items():
                with open(os.path.join(d, name), "w") as f:
                    f.write(text)
            r = subprocess.run(["CCJ"] + case["argv"], executable=REF, input=case["stdin"], capture_output=True,
                               text=True, cwd=d, timeout=600)
        rec = dict(case, rc=r.returncode, stdout=r.stdout, stderr=r.stderr)
        # anything that printed "SEQ\nSTRUCT (E)" went through the fill
        rec["fold"] = case["fold"] or (r.returncode == 0 and r.stdout.rstrip().endswith(")"))
        out.append(rec)
        print(case["argv"], r.returncode, repr((r.stdout + r.stderr)[:90]))
    with open(OUT, "w") as f:
        json.dump({"generator": "oracle/gen_cli_golden.py", "argv0": "CCJ", "cases": out}, f, indent=1)


if __name__ == "__main__":
    main()
