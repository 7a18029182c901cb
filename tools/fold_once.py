"""One n-nt fold (seed 5, Turner04) for profiler passes: python tools/fold_once.py [n] [folds]"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ccj_amd import W_final  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
r = random.Random(5)
wf = W_final("".join(r.choice("ACGU") for _ in range(n)), 2, params="Turner04")
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 1):
    e = wf.ccj()
print(n, e, wf.timing()["fill_ms"])
wf.close()
