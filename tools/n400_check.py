"""n=400 (BASELINE config 5 size) fold with and without split-point sharing: same MFE, structure and
W array (a size-independent property; full matrix hashes would need the 47 GB on the host)."""
import random
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ccj_amd import W_final  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
r = random.Random(6)
seq = "".join(r.choice("ACGU") for _ in range(n))
res = []
for kw in ({}, {"share_splits": -1}):
    t0 = time.time()
    wf = W_final(seq, 2, params="Turner04", **kw)
    e = wf.ccj()
    e = wf.ccj()
    res.append((e, wf.structure, [wf.W(j) for j in range(n + 1)]))
    print(kw, "mfe", e, "fill_ms", round(wf.timing()["fill_ms"], 1), "wall_s", round(time.time() - t0, 1), flush=True)
    print(wf.structure, flush=True)
    wf.close()
print("identical", res[0] == res[1], flush=True)
