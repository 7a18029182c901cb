#!/usr/bin/env python3
"""oracle/gen_traceback_n400.py — TEST INFRASTRUCTURE: the expected traceback outcome of every config-5
(n=400) sequence, for tests/test_gpu_configs.py::test_config5_batch400 (allow the reference's
impossible-case exit only where it is expected, and pin the structure everywhere else).

The oracle restatement (oracle/ccj_oracle.c) fills matrices but has no traceback, and a reference fold at
n=400 takes ~12 h (its stock build aborts at n >= 214), so the outcome comes from the host restatement of
the reference backtrack (ccj_host.cc Backtracker: W_final.cc:175-719 and pseudo_loop.cc:861-2820 in the
reference's order, pinned against the reference's stdout / stderr / exit code on the 116 CLI goldens and
the n <= 230 reference folds): W_final(..., host_traceback=True).  It runs over matrices whose 31 hashes
and W(n) are first checked equal to tests/golden/hashes_n400.json, so the outcome is a function of the
restatement-pinned fixture alone.  Needs a GPU (the fill) and ~50 GB of host memory for the mirror:

    python oracle/gen_traceback_n400.py            # every seed of hashes_n400.json not yet recorded
writes tests/golden/traceback_n400.json: [{"seed", "tag", "structure", "energy"} or {"seed", "tag", "exit": {...}}]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ccj_amd import BacktrackExit, W_final  # noqa: E402

FIX = os.path.join(ROOT, "tests", "golden", "hashes_n400.json")
OUT = os.path.join(ROOT, "tests", "golden", "traceback_n400.json")


def main():
    cases = json.load(open(FIX))
    done = {c["seed"]: c for c in json.load(open(OUT))} if os.path.exists(OUT) else {}
    for case in cases:
        if case["seed"] in done and "--redo" not in sys.argv:
            continue
        t0 = time.time()
        wf = W_final(case["seq"], case["dangles"], params=case["params"], noGU=bool(case["noGU"]), host_traceback=True)
        try:
            wf.fill()
            rec = {"seed": case["seed"], "tag": case["tag"],
                   "source": "ccj_host.cc host restatement of the reference backtrack over matrices equal to hashes_n400.json"}
            try:
                e = wf.result()  # W (host mode: computed here) and the traceback
                rec.update(structure=wf.structure, energy=e, stdout_msgs=wf.stdout_msgs)
            except BacktrackExit as ex:
                rec["exit"] = {"code": ex.exit_code, "msg": ex.msg, "stdout_msgs": ex.stdout}
            got = wf.hashes()
            bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
            if bad or wf.W(case["n"]) != case["mfe"]:
                raise SystemExit(f"seed {case['seed']}: matrices differ from hashes_n400.json ({bad}); nothing recorded")
        finally:
            wf.close()
        done[case["seed"]] = rec
        print(case["tag"], "exit" if "exit" in rec else rec["energy"], "%.1f s" % (time.time() - t0), flush=True)
        with open(OUT, "w") as f:
            json.dump([done[s] for s in sorted(done)], f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
