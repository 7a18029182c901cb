#!/usr/bin/env python3
"""oracle/gen_golden.py — TEST INFRASTRUCTURE: generate the committed golden fixtures.

Runs the real reference (oracle/_ref/ref_driver, compiled from /root/reference by
oracle/Makefile) in THIS container and records its outputs as data:

  tests/golden/e2e.json     (seq, params, dangles, noGU) -> reference stdout / stderr / exit code
                            of W_final(seq,dangle).ccj() printed exactly as src/CCJ.cc:107-108
  tests/golden/hashes.json  (seq, params, dangles, noGU) -> FNV-1a hash of every DP matrix after
                            the fill (canonical (i,j,k,l) order) + MFE (W[n])

Parameters are passed with --blob (our dump of the reference's scaled tables), and the script
first checks that --blob and -P <file>.par give identical hashes, so the blobs are pinned too.
The reference never leaves this container; only these JSON data files are committed.
"""
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
PARDIR = "/root/reference/params"
BLOBDIR = os.path.join(ROOT, "ccj_amd", "params")
OUT = os.path.join(ROOT, "tests", "golden")

TRNA32 = "GCGGAUUUAGCUCAGUUGGGAGAGCGCCAGAC"
CONDA = "GCAACGAUGACAUACAUCGCUAGUCGACGC"
PARFILES = {"Turner04": "rna_Turner04.par", "DirksPierce09": "rna_DirksPierce09.par",
            "DirksPierce03": "rna_DirksPierce03.par", "CaoChen06": "rna_CaoChen06.par",
            "CaoChen09": "rna_CaoChen09.par", "Matthews04": "dna_Matthews04.par"}


def rseq(seed, n, alphabet="ACGU"):
    r = random.Random(seed)
    return "".join(r.choice(alphabet) for _ in range(n))


def run(mode, seq, params, dangles, noGU, use_par=False):
    cmd = [DRV, mode]
    if use_par:
        cmd += ["-P", os.path.join(PARDIR, PARFILES[params])]
    else:
        cmd += ["--blob", os.path.join(BLOBDIR, params + ".ccjp")]
    cmd += ["-d", str(dangles)] + (["--noGU"] if noGU else []) + [seq]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=3600)
    return r.returncode, r.stdout, r.stderr


def parse_hashes(stdout):
    h, mfe = {}, None
    for line in stdout.splitlines():
        p = line.split()
        if p and p[0] == "HASH":
            h[p[1]] = p[2]
        elif p and p[0] == "MFE":
            mfe = int(p[1])
    return h, mfe


def cases():
    c = []
    for p in ["Turner04", "DirksPierce09", "DirksPierce03", "CaoChen06", "CaoChen09"]:
        c.append((TRNA32, p, 2, 0))
    c += [(TRNA32, "Turner04", 0, 0), (TRNA32, "Turner04", 1, 0), (TRNA32, "Turner04", 2, 1)]
    c += [(CONDA, "DirksPierce09", 2, 0), (CONDA, "Turner04", 2, 0)]
    # CLI DNA path: 'T' kept with --noConv -> Mathews 2004 + noGU (CCJ.cc:88-90)
    c.append((TRNA32.replace("U", "T"), "DNA_Mathews2004", 2, 1))
    c.append((rseq(1, 32), "Turner04", 2, 0))
    c.append((rseq(2, 50), "Turner04", 2, 0))
    c.append((rseq(2, 50), "DirksPierce09", 2, 0))
    # edge sizes
    for s in ["A", "GC", "GAC", "GCAU", "GGGAAAUCC", "GGGGAAAACCCC", "AAAAAAAAAAAAAAAAAAAA",
              "GCGCGCGCGCGCGCGCGCGCGCGC", "CCCCCCCCCCCGGGGGGGGGGG", "GGGGGGAAGGGGGGGGAACCCCCCACCCCCCCC"]:
        c.append((s, "Turner04", 2, 0))
        c.append((s, "DirksPierce09", 1, 0))
    # random cases
    for seed in range(100, 170):
        r = random.Random(seed)
        n = r.randint(8, 72)
        s = rseq(seed * 7 + 1, n)
        c.append((s, r.choice(["Turner04", "DirksPierce09", "DirksPierce03", "CaoChen09"]),
                  r.choice([0, 1, 2]), 1 if r.random() < 0.2 else 0))
    # GC-rich / pseudoknot-prone motifs
    for seed in range(200, 212):
        r = random.Random(seed)
        n = r.randint(30, 64)
        c.append((rseq(seed, n, "GGCCAU"), r.choice(["Turner04", "DirksPierce09"]), r.choice([1, 2]), 0))
    return c


def main():
    if not os.path.exists(DRV):
        sys.exit("build the oracle first: make -C oracle")
    os.makedirs(OUT, exist_ok=True)
    # pin the blobs: -P <par> and --blob must give identical matrices
    for p in ["Turner04", "DirksPierce09", "DirksPierce03"]:
        a = run("hash", TRNA32, p, 2, 0, use_par=True)
        b = run("hash", TRNA32, p, 2, 0, use_par=False)
        assert a == b, f"blob {p} differs from {PARFILES[p]}"
    e2e, hashes = [], []
    for (s, p, d, g) in cases():
        rc, out, err = run("fold", s, p, d, g)
        e2e.append({"seq": s, "params": p, "dangles": d, "noGU": g, "rc": rc, "stdout": out, "stderr": err})
        if len(s) <= 56:
            rc2, out2, _ = run("hash", s, p, d, g)
            assert rc2 == 0
            h, mfe = parse_hashes(out2)
            hashes.append({"seq": s, "params": p, "dangles": d, "noGU": g, "hashes": h, "mfe": mfe})
        print(len(s), p, d, g, rc, out.strip().splitlines()[-1] if out.strip() else err.strip()[:60], flush=True)
    with open(os.path.join(OUT, "e2e.json"), "w") as f:
        json.dump(e2e, f, indent=0)
    with open(os.path.join(OUT, "hashes.json"), "w") as f:
        json.dump(hashes, f, indent=0)


if __name__ == "__main__":
    main()
