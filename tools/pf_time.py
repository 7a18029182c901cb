"""Time the partition-function fill (include/ccj_pf.h) on random sequences: python tools/pf_time.py N [N ...]"""
import random
import sys
import time

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccj_amd  # noqa: E402

for n in [int(x) for x in sys.argv[1:]] or [100]:
    r = random.Random(5)
    seq = "".join(r.choice("ACGU") for _ in range(n))
    t0 = time.perf_counter()
    pf = ccj_amd.W_final_pf(seq, params="DirksPierce09")
    t1 = time.perf_counter()
    e = pf.ccj_pf()
    t2 = time.perf_counter()
    e = pf.ccj_pf()
    t3 = time.perf_counter()
    print("n=%d create %.1f ms first %.1f ms fill %.1f ms (events %.1f ms) energy %r cells %d" %
          (n, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), pf.fill_ms(), e, ccj_amd.num_cells(n)), flush=True)
    pf.close()
