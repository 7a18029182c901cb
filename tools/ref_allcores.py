"""The reference CPU CCJ at the headline size on all host cores (VERDICT r4 "missing" 4): k
concurrent oracle/_ref/ref_driver folds (the reference's W_final::ccj compiled from its own
sources; single-threaded, so k processes are its all-cores form) of n-nt random RNAs, seeds
seed..seed+k-1 (seed 5 is the bench.py headline sequence), Turner04, dangles 2.  Prints a progress
line every 30 s (gpurun treats 3 silent minutes as a hang) and one JSON line at the end.
usage: python tools/ref_allcores.py [n] [k] [seed]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import host_cores, num_cells, rseq  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    k = int(sys.argv[2]) if len(sys.argv) > 2 else host_cores()
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    blob = os.path.join(ROOT, "ccj_amd", "params", "Turner04.ccjp")
    import threading
    t0 = time.perf_counter()
    procs = [subprocess.Popen([drv, "fold", "--blob", blob, "--time", rseq(seed + r, n)], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(k)]
    res = [None] * k

    def wait(r):  # each process's own wall time (a fold that ends in the reference's backtrack exit prints no TIME)
        out, err = procs[r].communicate()
        res[r] = (time.perf_counter() - t0, procs[r].returncode, out, err)

    th = [threading.Thread(target=wait, args=(r,), daemon=True) for r in range(k)]
    for x in th:
        x.start()
    while any(x.is_alive() for x in th):
        time.sleep(30)
        print(f"{time.perf_counter() - t0:.0f} s, {sum(r is not None for r in res)}/{k} done", flush=True)
    wall = time.perf_counter() - t0
    per, lines, exits = [], [], 0
    for r, (sec, rc, out, err) in enumerate(res):
        # rc 1 + "This should not have happened!" is the reference's own backtrack exit (A-B5, after
        # the whole fill): a complete fold for this measurement
        if rc != 0 and "This should not have happened" not in err:
            print(json.dumps({"error": f"seed {seed + r}: rc {rc}", "stderr": err[-500:]}))
            return 1
        exits += rc != 0
        per.append(sec)
        lines.append(out.strip().splitlines()[-1] if out.strip() else err.strip().splitlines()[-1])
    cells = num_cells(n)
    print(json.dumps({"n": n, "cores": k, "seeds": [seed, seed + k - 1], "params": "Turner04", "wall_s": wall,
                      "cells_per_fold": cells, "value": k * cells / wall, "unit": "DP-cells/s",
                      "per_process_seconds": {"min": min(per), "max": max(per), "first": per[0]},
                      "reference_backtrack_exits": exits,
                      "single_core_cells_per_s": cells / per[0], "seed%d_line" % seed: lines[0],
                      "what": "k concurrent reference folds (W_final::ccj incl. its constructor) on the GPU box's host"}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
