#!/usr/bin/env python3
"""oracle/gen_hashes_large.py — TEST INFRASTRUCTURE: full-matrix goldens at BASELINE sizes.

Runs the real reference (oracle/_ref/ref_driver fold --hash, compiled from /root/reference/src)
on the BASELINE.json configs' sequences and on sequences past the stock n >= 214 assert abort
(`ref_driver_ndebug`, the same sources built with -DNDEBUG, identical output for
n <= 213).  One run gives the CLI's two stdout lines (W_final::ccj(), CCJ.cc:104-108) and, after
the fold, one FNV-1a hash per DP matrix in canonical (i,j,k,l) order (all 22 Matrix4D, P, WBP,
WPP, V, Vtype, WM, WMv, WMp, W).  n=200 takes ~23 min of one core, n=220 ~40 min, so the runs are
started detached and collected later:

    python oracle/gen_hashes_large.py start    # one background process per case
    python oracle/gen_hashes_large.py collect  # writes tests/golden/hashes_large.json
"""
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
WORK = "/tmp/refhash"
# (tag, seed, n, params, reference .par, driver)
RUNS = [
    ("t04_100", 3, 100, "Turner04", "rna_Turner04.par", "ref_driver"),
    ("t04_150", 4, 150, "Turner04", "rna_Turner04.par", "ref_driver"),
    ("t04_200", 5, 200, "Turner04", "rna_Turner04.par", "ref_driver"),
    ("dp09_200", 5, 200, "DirksPierce09", "rna_DirksPierce09.par", "ref_driver"),
    ("t04_220", 7, 220, "Turner04", "rna_Turner04.par", "ref_driver_ndebug"),
    ("dp09_230", 8, 230, "DirksPierce09", "rna_DirksPierce09.par", "ref_driver_ndebug"),
]


def seq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


def start():
    os.makedirs(WORK, exist_ok=True)
    for tag, s, n, _, par, drv in RUNS:
        if os.path.exists(os.path.join(WORK, tag + ".out")):
            continue
        with open(os.path.join(WORK, tag + ".out"), "w") as o, open(os.path.join(WORK, tag + ".err"), "w") as e:
            subprocess.Popen([os.path.join(REF, drv), "fold", "-P", "/root/reference/params/" + par, "--time",
                              "--hash", seq(s, n)], stdout=o, stderr=e, start_new_session=True)
        print("started", tag)


def collect():
    out = []
    for tag, s, n, p, par, drv in RUNS:
        fo, fe = os.path.join(WORK, tag + ".out"), os.path.join(WORK, tag + ".err")
        if not os.path.exists(fo):
            continue
        lines = open(fo).read().splitlines()
        if not lines or not lines[-1].startswith("MFE "):
            print("not finished:", tag)
            continue
        err = open(fe).read()
        hashes = {ln.split()[1]: ln.split()[2] for ln in lines if ln.startswith("HASH ")}
        stdout = "".join(ln + "\n" for ln in lines if not ln.startswith(("HASH ", "MFE ")))
        out.append({"tag": tag, "seed": s, "n": n, "seq": seq(s, n), "params": p, "dangles": 2, "noGU": 0,
                    "driver": drv, "stdout": stdout, "hashes": hashes, "mfe": int(lines[-1].split()[1]),
                    "ref_seconds": float(err.split("TIME")[1].split()[0])})
    with open(os.path.join(ROOT, "tests", "golden", "hashes_large.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(out), "cases")


if __name__ == "__main__":
    {"start": start, "collect": collect}[sys.argv[1]]()
