"""Which matrices / cells of a GPU fold differ from the C oracle (debugging aid, -m gpu box).
usage: python tools/dbg_diff.py [n] [seed] [params] [shard_world]"""
import random
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ccj_amd import MAT4, W_final  # noqa: E402
from tests.oracle_lib import OracleFold, blob  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
params = sys.argv[3] if len(sys.argv) > 3 else "Turner04"
world = int(sys.argv[4]) if len(sys.argv) > 4 else 1
r = random.Random(seed)
seq = "GCGGAUUUAGCUCAGUUGGGAGAGCGCCAGAC" if n == 32 and seed == 0 else "".join(r.choice("ACGU") for _ in range(n))
kw = dict(shard_world=world, shard_simulate=True) if world > 1 else {}
wf = W_final(seq, 2, params=params, **kw)
wf.fill()
o = OracleFold(seq, blob(params), 2, 0)
hg, hc = wf.hashes(), o.hashes()
bad = [k for k in hg if hg[k] != hc[k]]
print("n", n, "seed", seed, "differ:", bad)
diffs = []
for name in bad:
    if name not in MAT4:
        continue
    x = MAT4.index(name)
    for i in range(1, n + 1):
        for j in range(i, n + 1):
            for k in range(j + 2, n + 1):
                for l in range(k, n + 1):
                    g, c = wf.get4(x, i, j, k, l), o.get4(x, i, j, k, l)
                    if g != c:
                        diffs.append((j - i + l - k, name, i, j, k, l, g, c))
diffs.sort()
for t, name, i, j, k, l, g, c in diffs[:25]:
    print(f"  t={t} {name}({i},{j},{k},{l}) a={j-i} b={l-k} h={k-j-2}: gpu {g} oracle {c}")
print("total differing cells", len(diffs))
