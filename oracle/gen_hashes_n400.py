#!/usr/bin/env python3
"""oracle/gen_hashes_n400.py — TEST INFRASTRUCTURE: the config-5 (n=400) matrix fixture.

A reference fold at n=400 takes ~12 h of one core (and the stock build aborts at n >= 214,
matrices.hh:159-160), so config 5 is pinned by the C restatement instead: oracle/ccj_oracle.c's
level-parallel mode (ccj_oracle_fold_par, OpenMP), whose equality with the reference is checked on
every reference fixture up to n=230 (tests/test_oracle.py).  This fixture is therefore
"restatement-pinned, not a reference run".  It holds all 31 matrix hashes (FNV-1a, canonical order,
the ref_driver convention) and W[n] for BASELINE config 5's first sequence: random.Random(6), 400 nt,
rna_Turner04, dangles 2 (bench.py --n 400 --seed 6).  Needs ~49 GB of RAM and ~2-3 h on 8 cores:

    nohup python oracle/gen_hashes_n400.py > /tmp/n400.log 2>&1 &
"""
import ctypes
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.oracle_lib import HASH_NAMES, blob, oracle_lib  # noqa: E402

# Config 5 is seeds 6..13 (bench.py --n 400 --seed 6 --gpus 8: rank r folds seed 6 + r).
CASES = [("t04_400_seed%d" % s, s, 400, "Turner04") for s in range(6, 14)]


def seq(seed, n):
    r = random.Random(seed)
    return "".join(r.choice("ACGU") for _ in range(n))


def main():
    """python oracle/gen_hashes_n400.py [tag ...]: (re)computes the named cases (default: all) and
    keeps the other cases already in the fixture."""
    L = oracle_lib()
    os.environ["CCJ_ORACLE_PROGRESS"] = "1"
    out_path = os.path.join(ROOT, "tests", "golden", "hashes_n400.json")
    want = sys.argv[1:] or [c[0] for c in CASES]
    out = []
    if os.path.exists(out_path):
        with open(out_path) as f:
            out = [c for c in json.load(f) if c["tag"] not in want]
    nthr = int(os.environ.get("CCJ_ORACLE_THREADS", "0")) or os.cpu_count() or 8
    for tag, s, n, params in CASES:
        if tag not in want:
            continue
        b = ctypes.create_string_buffer(blob(params))
        t0 = time.time()
        h = L.ccj_oracle_fold_par(seq(s, n).encode(), b, 2, 0, nthr)
        if not h:
            raise MemoryError("oracle allocation failed")
        t1 = time.time()
        hv = (ctypes.c_uint64 * 31)()
        L.ccj_oracle_hashes(h, hv)
        out.append({"tag": tag, "seed": s, "n": n, "seq": seq(s, n), "params": params, "dangles": 2, "noGU": 0,
                    "source": "oracle/ccj_oracle.c ccj_oracle_fold_par (restatement-pinned, not a reference run)",
                    "hashes": {HASH_NAMES[i]: "%016x" % hv[i] for i in range(31)},
                    "mfe": L.ccj_oracle_W(h, n), "oracle_seconds": t1 - t0, "threads": nthr})
        L.ccj_oracle_free(h)
        print(tag, "done in %.0f s, mfe %d" % (t1 - t0, out[-1]["mfe"]), flush=True)
        # Merge with the file as it is now: other fields (e.g. the traceback outcome) may have been
        # added to the other cases while this fold ran.
        if os.path.exists(out_path):
            with open(out_path) as f:
                disk = {c["tag"]: c for c in json.load(f)}
            mine = {c["tag"] for c in out if c["tag"] in want}
            out = [c for c in out if c["tag"] in mine] + [c for t, c in disk.items() if t not in mine]
        out.sort(key=lambda c: c["seed"])
        with open(out_path, "w") as f:
            json.dump(out, f, indent=1)
    print("wrote", out_path)


if __name__ == "__main__":
    main()
