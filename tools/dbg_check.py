"""Run the bounds-checked debug build over small folds (every 4-D / 2-D / e_intP index is
validated on the device; a violation sets a flag instead of touching memory)."""
import os
import random
import sys

os.environ["CCJ_LIB_VARIANT"] = "dbg"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ccj_amd import W_final  # noqa: E402

for n in [1, 2, 3, 4, 5, 6, 7, 8, 12, 20, 33, 47, 64, 90]:
    r = random.Random(n)
    s = "".join(r.choice("ACGU") for _ in range(n))
    # split_target -1: no split levels, so split-point sharing covers every level
    for params, st in [("Turner04", 0), ("DirksPierce09", 0), ("Turner04", -1)]:
        wf = W_final(s, 2, params=params, split_target=st)
        wf.fill()
        try:
            e = wf.result()
            print(n, params, st, wf.structure, e, wf.timing()["fill_ms"], flush=True)
        except Exception as ex:
            print(n, params, "backtrack exit:", ex, flush=True)
        wf.close()
print("DBG_OK")
