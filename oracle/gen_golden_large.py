#!/usr/bin/env python3
"""oracle/gen_golden_large.py — TEST INFRASTRUCTURE: end-to-end goldens at BASELINE sizes.

Runs the real reference (oracle/_ref/ref_driver fold, -P <reference .par>) on the BASELINE.json
configs' sequences — random.Random(seed).choice('ACGU') x n — and records stdout/stderr/rc plus
the single-core wall time.  n=200 takes ~22 min per fold, so the runs are started in the
background into a work directory and this script collects whatever has finished:

    python oracle/gen_golden_large.py start   # launches the reference runs (one core each)
    python oracle/gen_golden_large.py collect # writes tests/golden/e2e_large.json
"""
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
WORK = "/tmp/refruns"
RUNS = [  # (tag, seed, n, params, parfile)
    ("t04_100", 3, 100, "Turner04", "rna_Turner04.par"),
    ("t04_150", 4, 150, "Turner04", "rna_Turner04.par"),
    ("t04_200", 5, 200, "Turner04", "rna_Turner04.par"),
    ("dp09_200", 5, 200, "DirksPierce09", "rna_DirksPierce09.par"),
]


def seq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


def start():
    os.makedirs(WORK, exist_ok=True)
    for tag, s, n, _, par in RUNS:
        if os.path.exists(os.path.join(WORK, tag + ".out")):
            continue
        with open(os.path.join(WORK, tag + ".out"), "w") as o, open(os.path.join(WORK, tag + ".err"), "w") as e:
            subprocess.Popen([DRV, "fold", "-P", "/root/reference/params/" + par, "--time", seq(s, n)],
                             stdout=o, stderr=e, start_new_session=True)


def collect():
    out = []
    for tag, s, n, p, par in RUNS:
        fo, fe = os.path.join(WORK, tag + ".out"), os.path.join(WORK, tag + ".err")
        if not os.path.exists(fe):
            continue
        err = open(fe).read()
        if "TIME" not in err:
            print("not finished:", tag)
            continue
        t = float(err.split("TIME")[1].split()[0])
        out.append({"tag": tag, "seed": s, "n": n, "seq": seq(s, n), "params": p, "dangles": 2, "noGU": 0,
                    "rc": 0, "stdout": open(fo).read(), "stderr": err.split("TIME")[0], "ref_seconds": t})
    with open(os.path.join(ROOT, "tests", "golden", "e2e_large.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(out), "cases")


if __name__ == "__main__":
    {"start": start, "collect": collect}[sys.argv[1]]()
