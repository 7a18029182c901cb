#!/usr/bin/env python3
"""oracle/gen_pf_golden.py — TEST INFRASTRUCTURE: golden vectors for the partition function (f4).

Runs the reference's W_final_pf (src/part_func.cc + stoch_backtrack.cc, compiled by
oracle/Makefile into oracle/_ref/pf_driver with -ffp-contract=off) on synthetic sequences and
records, as data, in tests/golden/pf_golden.json:

  {"name", "seq", "params", "dangles", "energy" (repr of the double), "wbits" (IEEE bits of
   W[0..n]), "h2" {2-D matrix: FNV-1a of its IEEE bits}, "h4" {4-D matrix: FNV-1a of its int32
   values}, "exp" {Boltzmann table: FNV-1a}, optionally "srand" + "samples" (5 Sample_W(1, n)
   after srand(seed); + "sample_exit", the line the reference printed before exit(0))}

Parameter sets: "default" = the reference's compiled-in Turner 2004 tables (no -P), otherwise
-P /root/reference/params/rna_<name>.par.  The reference never leaves this container; only these
numbers travel.  Usage: python3 oracle/gen_pf_golden.py [--jobs 8] [--big]
       python3 oracle/gen_pf_golden.py --large   (tests/golden/pf_golden_large.json: the bench.py --pf
       sequence, n=200 seed 5 with rna_Turner04.par, and n=150; about an hour of reference time)
"""
import argparse
import json
import os
import random
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(ROOT, "oracle", "_ref", "pf_driver")
PARDIR = "/root/reference/params"
OUT = os.path.join(ROOT, "tests", "golden", "pf_golden.json")
OUT_LARGE = os.path.join(ROOT, "tests", "golden", "pf_golden_large.json")


def rseq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


def cases(big):
    out = []
    # edge sizes, both parameter sets, every dangles model
    for n in (1, 2, 3, 4, 5, 6, 8):
        out.append(("edge%d" % n, rseq(100 + n, n), "default", 2, None))
    for n in (12, 16, 20, 25, 30):
        for params in ("default", "DirksPierce09"):
            for d in (0, 1, 2):
                out.append(("r%d_%s_d%d" % (n, params, d), rseq(200 + n, n), params, d, None))
    # special hairpins (tetra/tri/hexa loops of Turner 2004) and helices long enough to overflow
    # the int 4-D cells (the x86 truncation path)
    for name, s in (("tetra", "GGGGCGAAAGCCCCAUAUGGGGCGAAAGCCCC"), ("tri", "GGGCAACGCCCAGGCAACGCCUU"),
                    ("hexa", "GGGACAUGGAGUCCCAAGGGACAUGGAGUCCC"), ("helix", "GGGGGGGGGGAAAACCCCCCCCCCAAAGGGGGCCCCC"),
                    ("knot", "GGGGAAAACCCCGGGGAAAACCCCGGGGUUUUCCCCAAAAGGGG")):
        for params in ("default", "DirksPierce09"):
            out.append(("%s_%s" % (name, params), s, params, 2, None))
    # larger random sequences, with stochastic samples
    for n, seed in ((40, 1), (50, 2), (60, 3)):
        for params in ("default", "DirksPierce09"):
            out.append(("big%d_%s" % (n, params), rseq(seed, n), params, 2, seed))
    for name, s, params in (("samp_tetra", "GGGGCGAAAGCCCCAUAUGGGGCGAAAGCCCC", "DirksPierce09"),
                            ("samp_helix", "GGGGGGGGGGAAAACCCCCCCCCCAAAGGGGGCCCCC", "default"),
                            ("samp_r30", rseq(230, 30), "default")):
        for seed in (1, 7, 12345):
            out.append(("%s_s%d" % (name, seed), s, params, 2, seed))
    if big:
        out.append(("big80_default", rseq(8, 80), "default", 2, 3))
        out.append(("big100_DirksPierce09", rseq(9, 100), "DirksPierce09", 2, 5))
    return out


def large_cases():
    # bench.py --pf's default workload (rseq(5, 200), Turner04, dangles 2) and a second size/set
    return [("pf200_Turner04_seed5", rseq(5, 200), "Turner04", 2, None),
            ("pf150_DirksPierce09_seed4", rseq(4, 150), "DirksPierce09", 2, 11)]


def run(case):
    name, seq, params, dangles, xs = case
    cmd = [DRV, seq, "-d", str(dangles)]
    if params != "default":
        cmd += ["-P", os.path.join(PARDIR, "rna_%s.par" % params)]
    if xs:
        cmd += ["--samples", "5", "--srand", str(xs)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=4 * 3600)
    if p.returncode != 0:
        raise RuntimeError("%s: rc %d %s" % (name, p.returncode, p.stderr[-400:]))
    rec = {"name": name, "seq": seq, "params": params, "dangles": dangles, "h2": {}, "h4": {}, "exp": {}}
    samples, tail = [], []
    for line in p.stdout.splitlines():
        w = line.split()
        if not w:
            continue
        if w[0] == "ENERGY":
            rec["energy"] = w[1]
        elif w[0] == "WBITS":
            rec["wbits"] = w[1:]
        elif w[0] == "H2":
            rec["h2"][w[1]] = w[2]
        elif w[0] == "H4":
            rec["h4"][w[1]] = w[2]
        elif w[0] == "EXP":
            rec["exp"][w[1]] = w[2]
        elif w[0] == "SAMPLE":
            samples.append(w[1] if len(w) > 1 else "")
        else:
            tail.append(line)
    if xs:
        rec["srand"] = xs
        rec["samples"] = samples
        if len(samples) < 5:
            rec["sample_exit"] = "\n".join(tail) + "\n"
    return rec


SETS = {"default": [], "Turner04": ["-P", PARDIR + "/rna_Turner04.par"],
        "DirksPierce09": ["-P", PARDIR + "/rna_DirksPierce09.par"], "DirksPierce03": ["-P", PARDIR + "/rna_DirksPierce03.par"],
        "CaoChen06": ["-P", PARDIR + "/rna_CaoChen06.par"], "CaoChen09": ["-P", PARDIR + "/rna_CaoChen09.par"],
        "Matthews04": ["-P", PARDIR + "/dna_Matthews04.par"], "DNA_Mathews2004": ["--dna"]}


def exp_tables():
    """The Boltzmann-table hashes of every bundled parameter set (a 9-nt run of each)."""
    out = {}
    for name, args in SETS.items():
        p = subprocess.run([DRV, "GGGAAACCC"] + args, capture_output=True, text=True, timeout=600)
        out[name] = {w[1]: w[2] for w in (l.split() for l in p.stdout.splitlines()) if w and w[0] == "EXP"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--large", action="store_true")
    a = ap.parse_args()
    if a.large:
        with ThreadPoolExecutor(2) as ex:
            recs = list(ex.map(run, large_cases()))
        with open(OUT_LARGE, "w") as f:
            json.dump({"generator": "oracle/gen_pf_golden.py --large",
                       "driver": "oracle/_ref/pf_driver (part_func.cc, -ffp-contract=off)", "cases": recs}, f, indent=0)
        print("wrote %d cases to %s" % (len(recs), OUT_LARGE))
        return 0
    cs = cases(a.big)
    with ThreadPoolExecutor(a.jobs) as ex:
        recs = list(ex.map(run, cs))
    with open(OUT, "w") as f:
        json.dump({"generator": "oracle/gen_pf_golden.py", "driver": "oracle/_ref/pf_driver (part_func.cc, -ffp-contract=off)",
                   "exp_sets": exp_tables(), "cases": recs}, f, indent=0)
    print("wrote %d cases to %s" % (len(recs), OUT))


if __name__ == "__main__":
    sys.exit(main())
