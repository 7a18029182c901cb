"""The interior-loop work decomposition checked against the reference (-m gpu): the k_iloop work
items (ccj_items.h, 128-cell items), counted two ways, each unsharded and band-sharded.

In items mode ccj_reset sizes the k_iloop launches from per-(level, shard, split) item counts made
on the GPU by k_items; the host holds the same enumeration twice (count_level_items, the fast row walk, and
the generic item_row).  With CCJ_CHECK_ITEMS=1 every reset recomputes both on the host and fails
with CCJ_E_STATE if either disagrees with the GPU's count; CCJ_HOST_COUNT=1 sizes the launches from
the host count alone.  The switches are read once per process, so each mode runs in a child
interpreter that folds reference cases (unsharded and band-sharded in one context) and prints every
matrix hash; the parent compares them with the reference's (tests/golden/hashes_large.json).
"""
import json
import os
import subprocess
import sys

import pytest

from tests.oracle_lib import golden

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [c for c in golden("hashes_large.json") if c["n"] in (100, 150)]

CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from ccj_amd import W_final
out = []
for case in json.loads(sys.argv[2]):
    for world in (1, 4):
        kw = {} if world == 1 else dict(shard_world=world, shard_simulate=True)
        wf = W_final(case["seq"], case["dangles"], params=case["params"], noGU=bool(case["noGU"]), **kw)
        try:
            e = wf.ccj()
            out.append({"tag": case["tag"], "world": world, "hashes": wf.hashes(), "line": f"{wf.structure} ({e:g})"})
        finally:
            wf.close()
print(json.dumps(out))
"""


@pytest.mark.parametrize("mode", [{"CCJ_CHECK_ITEMS": "1"},
                                  {"CCJ_HOST_COUNT": "1", "CCJ_CHECK_ITEMS": "1"}],
                         ids=["items-gpu-count-checked", "items-host-count"])
def test_item_counts_agree_and_fold_matches_reference(mode):
    env = dict(os.environ, **mode)
    cases = [{k: c[k] for k in ("tag", "seq", "dangles", "params", "noGU")} for c in CASES]
    p = subprocess.run([sys.executable, "-c", CHILD, ROOT, json.dumps(cases)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    got = json.loads(p.stdout.strip().splitlines()[-1])
    assert len(got) == 2 * len(CASES)
    by_tag = {c["tag"]: c for c in CASES}
    for r in got:
        case = by_tag[r["tag"]]
        bad = [k for k in case["hashes"] if r["hashes"][k] != case["hashes"][k]]
        assert not bad, f"{r['tag']} world {r['world']}: matrices differ from the reference: {bad}"
        assert r["line"] == case["stdout"].splitlines()[-1]
