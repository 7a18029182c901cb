"""Per-level kernel times of one n-nt fold (HIP events on the fill stream)."""
import ctypes
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ccj_amd import W_final, lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
SEED = int(os.environ.get("CCJ_PROFILE_SEED", "5"))
r = random.Random(SEED)
seq = "".join(r.choice("ACGU") for _ in range(n))
wf = W_final(seq, 2, params="Turner04")
wf.ccj()
fills = []
for _ in range(int(os.environ.get("CCJ_PROFILE_REPS", "5"))):
    wf.ccj()
    fills.append(wf.timing()["fill_ms"])
lev1 = wf.timing()["level4d_ms"]
if os.environ.get("CCJ_PROFILE_DUMP"):
    # every level's span on the level stream in the last uninstrumented fold (lev_done[t-1] -> lev_done[t]:
    # the level chain's critical path, waits included), for tools/shard_projection.py
    _L = lib()
    _L.ccj_level_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    _lv = (ctypes.c_double * n)()
    _L.ccj_level_times(wf._h, _lv, None, n)
    with open(os.environ["CCJ_PROFILE_DUMP"], "w") as f:
        json.dump({"n": n, "seed": SEED, "params": "Turner04", "fill_ms": fills[-1], "level_ms": list(_lv)[:n - 2]}, f)
# one more fold with a marker pair around every launch for the per-kernel breakdown (slower fill)
wf.set_timing(2)
wf.ccj()
L = lib()
L.ccj_level_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int]
lv = (ctypes.c_double * n)()
dg = (ctypes.c_double * n)()
L.ccj_level_times(wf._h, lv, dg, n)
il = (ctypes.c_double * n)()
L.ccj_iloop_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
L.ccj_iloop_times(wf._h, il, n)
tm = wf.timing()
tm["fill_ms_median"] = sorted(fills)[len(fills) // 2]
tm["fill_ms_min"] = min(fills)
tm["fill_ms_instrumented"] = tm.pop("fill_ms")
tm["level4d_ms_uninstrumented"] = lev1
print(json.dumps(tm))
for t in range(0, n, max(1, n // 25)):
    print(f"t={t:4d} level4d {lv[t]*1e3:9.1f} us   iloop {il[t]*1e3:8.1f} us   diag2d {dg[t]*1e3:8.1f} us")
print("sum level", sum(lv), "sum iloop", sum(il), "sum diag", sum(dg))
