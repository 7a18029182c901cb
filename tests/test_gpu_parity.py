"""GPU parity tests (-m gpu, MI355X): the HIP fill + host backtrack against the reference.

  * every DP matrix (22 four-dimensional + 8 two-dimensional + W) bit-identical to the real
    reference's fill (tests/golden/hashes.json, from oracle/_ref/ref_driver),
  * end-to-end CLI output identical to the reference (tests/golden/e2e.json: stdout incl.
    "Should not be here!" lines, stderr, exit codes of the reference's backtrack exits),
  * fresh random inputs against the C restatement (oracle/ccj_oracle.c), bit-exact,
  * BASELINE sizes (n = 100 / 150 / 200) against the reference's own outputs
    (tests/golden/e2e_large.json) plus size-independent properties (determinism, overlapped vs
    synchronous host mirror, MFE == W[n] / 100).
Everything calls through the C ABI of libccj_hip.so; nothing here falls back to the CPU.
"""
import random

import pytest

from tests.oracle_lib import OracleFold, blob, golden

pytestmark = pytest.mark.gpu

HASHES = golden("hashes.json")
E2E = golden("e2e.json")


def _wf(seq, params, dangles, noGU, **kw):
    from ccj_amd import W_final
    return W_final(seq, dangles, params=params, noGU=bool(noGU), **kw)


@pytest.mark.parametrize("case", HASHES, ids=lambda c: f"n{len(c['seq'])}-{c['params']}-d{c['dangles']}-g{c['noGU']}")
def test_matrices_bit_identical_to_reference(case):
    wf = _wf(case["seq"], case["params"], case["dangles"], case["noGU"])
    try:
        wf.fill()
        try:
            wf.result()
        except Exception:
            pass  # some references exit in the backtrack; W is computed before it
        got = wf.hashes()
        bad = [k for k in case["hashes"] if got[k] != case["hashes"][k]]
        assert not bad, f"matrices differ from the reference: {bad}"
        assert wf.W(len(case["seq"])) == case["mfe"]
    finally:
        wf.close()


@pytest.mark.parametrize("case", E2E, ids=lambda c: f"n{len(c['seq'])}-{c['params']}-d{c['dangles']}-g{c['noGU']}")
def test_cli_output_identical_to_reference(case):
    from ccj_amd.cli import fold_cli
    rc, out, err = fold_cli(case["seq"], case["params"], case["dangles"], bool(case["noGU"]))
    assert out == case["stdout"]
    assert rc == case["rc"]
    assert err == case["stderr"]


def _rseq(seed, n, alphabet="ACGU"):
    r = random.Random(seed)
    return "".join(r.choice(alphabet) for _ in range(n))


@pytest.mark.parametrize("seed", range(8))
def test_random_inputs_match_oracle(seed):
    r = random.Random(1000 + seed)
    n = r.randint(20, 60)
    seq = _rseq(5000 + seed, n, r.choice(["ACGU", "GGCCAU", "GCAU"]))
    params = r.choice(["Turner04", "DirksPierce09", "DirksPierce03", "CaoChen09", "Matthews04"])
    d, g = r.choice([0, 1, 2]), r.random() < 0.25
    o = OracleFold(seq, blob(params), d, int(g))
    wf = _wf(seq, params, d, g)
    try:
        wf.fill()
        try:
            wf.result()
        except Exception:
            pass
        assert wf.hashes() == o.hashes()
    finally:
        wf.close()
        o.close()


@pytest.mark.parametrize("case", golden("e2e_large.json"), ids=lambda c: c["tag"])
def test_baseline_sizes_match_reference(case):
    from ccj_amd.cli import fold_cli
    rc, out, err = fold_cli(case["seq"], case["params"], case["dangles"], bool(case["noGU"]))
    assert (rc, out, err) == (case["rc"], case["stdout"], case["stderr"])


def test_determinism_and_mirror_modes():
    """Size-independent properties at a larger n: two fills are identical, and the overlapped
    level-by-level D2H mirror equals a synchronous full copy."""
    seq = _rseq(77, 120)
    a = _wf(seq, "Turner04", 2, 0, overlap_d2h=True)
    b = _wf(seq, "Turner04", 2, 0, overlap_d2h=False)
    try:
        a.fill()
        ea = a.result()
        ha = a.hashes()
        a.fill()
        a.result()
        assert a.hashes() == ha
        b.fill()
        eb = b.result()
        assert b.hashes() == ha
        assert ea == eb == a.W(120) / 100.0
        assert a.structure == b.structure and len(a.structure) == 120
    finally:
        a.close()
        b.close()


def _result(wf):
    from ccj_amd import BacktrackExit
    try:
        e = wf.result()
        return ("ok", e, wf.structure, wf.stdout_msgs)
    except BacktrackExit as ex:
        return ("exit", ex.exit_code, ex.msg, ex.stdout)


@pytest.mark.parametrize("seed", range(12))
def test_device_traceback_equals_host_traceback(seed):
    """The GPU traceback (ccj_backtrack.hip, wave-parallel first-minimum scans) and the host
    restatement over the mirror give the same MFE, brackets, stdout lines and exits."""
    r = random.Random(7000 + seed)
    n = r.choice([24, 40, 64, 90, 130])
    seq = _rseq(9000 + seed, n, r.choice(["ACGU", "GGCCAU", "GCAU"]))
    params = r.choice(["Turner04", "DirksPierce09", "DirksPierce03", "CaoChen09", "Matthews04"])
    d, g = r.choice([0, 1, 2]), r.random() < 0.25
    dev = _wf(seq, params, d, g)
    host = _wf(seq, params, d, g, host_traceback=True, overlap_d2h=True)
    try:
        dev.fill()
        host.fill()
        assert _result(dev) == _result(host)
        assert [dev.W(j) for j in range(n + 1)] == [host.W(j) for j in range(n + 1)]
    finally:
        dev.close()
        host.close()


@pytest.mark.parametrize("case", [c for c in E2E if len(c["seq"]) >= 30][:20],
                         ids=lambda c: f"n{len(c['seq'])}-{c['params']}-d{c['dangles']}-g{c['noGU']}")
def test_host_traceback_matches_reference(case):
    """The host restatement (mirror path) against the reference's CLI output, so both traceback
    implementations stay pinned."""
    wf = _wf(case["seq"], case["params"], case["dangles"], case["noGU"], host_traceback=True)
    try:
        wf.fill()
        res = _result(wf)
        last = case["stdout"].splitlines()[-1] if case["stdout"] else ""
        if res[0] == "ok":
            assert f"{res[2]} ({res[1]:g})" == last
        else:
            assert res[1] == case["rc"] and res[2] == case["stderr"]
    finally:
        wf.close()


FUZZ = int(__import__("os").environ.get("CCJ_FUZZ", "0"))


@pytest.mark.skipif(FUZZ <= 0, reason="opt-in randomized campaign: CCJ_FUZZ=<cases> (seconds to a minute per case)")
@pytest.mark.parametrize("k", range(max(FUZZ, 1)))
def test_fuzz_random_folds(k):
    """Opt-in randomized parity campaign (round 6): a random sequence (n 20-110, alphabet, parameter
    set, dangles, noGU) folded on the GPU must give the restatement's 31 matrix hashes (both fill
    modes of the oracle are pinned against the reference in tests/test_oracle.py), and the device
    traceback must give the host restatement's structure, energy, side messages or exit."""
    r = random.Random(90000 + k)
    n = r.randint(20, 110)
    seq = _rseq(91000 + k, n, r.choice(["ACGU", "ACGU", "GGCCAU", "GCAU", "AU"]))
    params = r.choice(["Turner04", "DirksPierce09", "DirksPierce03", "CaoChen09", "Matthews04"])
    d, g = r.choice([0, 1, 2]), r.random() < 0.25
    o = OracleFold(seq, blob(params), d, int(g), threads=0)
    dev = _wf(seq, params, d, g)
    host = _wf(seq, params, d, g, host_traceback=True)
    try:
        dev.fill()
        rd = _result(dev)
        assert dev.hashes() == o.hashes(), (n, params, d, g)
        host.fill()
        assert _result(host) == rd, (n, params, d, g)
    finally:
        dev.close()
        host.close()
        o.close()


REF_FUZZ = int(__import__("os").environ.get("CCJ_REF_FUZZ", "0"))
REF_DRV = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))),
                                     "oracle", "_ref", "ref_driver")


@pytest.mark.skipif(REF_FUZZ <= 0 or not __import__("os").path.exists(REF_DRV),
                    reason="opt-in randomized campaign against the reference's own build: CCJ_REF_FUZZ=<cases>")
def test_fuzz_against_reference_driver():
    """Opt-in randomized campaign (round 6) against the real reference: random sequences (n 10-70, or up
    to CCJ_REF_FUZZ_NMAX,
    three alphabets, four parameter sets, dangles 0/1/2, noGU) through oracle/_ref/ref_driver (the
    reference's own fill, built here from its sources; 16 at a time on the host) and through the GPU:
    all 31 matrix hashes and W(n) identical."""
    import concurrent.futures
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cases = []
    for k in range(REF_FUZZ):
        r = random.Random(80000 + k)
        n = r.randint(10, int(os.environ.get("CCJ_REF_FUZZ_NMAX", "70")))
        seq = _rseq(81000 + k, n, r.choice(["ACGU", "GGCCAU", "GCAU"]))
        cases.append((seq, r.choice(["Turner04", "DirksPierce09", "DirksPierce03", "CaoChen09"]), r.choice([0, 1, 2]),
                      r.random() < 0.25))

    def ref(c):
        seq, params, d, g = c
        cmd = [REF_DRV, "hash", "--blob", os.path.join(root, "ccj_amd", "params", params + ".ccjp"), "-d", str(d)]
        p = subprocess.run(cmd + (["--noGU"] if g else []) + [seq], capture_output=True, text=True, timeout=600)
        h, mfe = {}, None
        for line in p.stdout.splitlines():
            w = line.split()
            if w and w[0] == "HASH":
                h[w[1]] = w[2]
            elif w and w[0] == "MFE":
                mfe = int(w[1])
        return p.returncode, h, mfe

    refs = [None] * len(cases)
    with concurrent.futures.ThreadPoolExecutor(16) as ex:
        futs = {ex.submit(ref, c): i for i, c in enumerate(cases)}
        for done, f in enumerate(concurrent.futures.as_completed(futs), 1):
            refs[futs[f]] = f.result()
            if done % 16 == 0:
                print(f"reference folds done: {done}/{len(cases)}", flush=True)
    bad = []
    for c, (rc, h, mfe) in zip(cases, refs):
        assert rc == 0 and len(h) == 31, c
        wf = _wf(*c)
        try:
            wf.fill()
            try:
                wf.result()  # W is computed here (before any backtrack exit of the reference's)
            except Exception:
                pass
            got = wf.hashes()
            if any(got[x] != h[x] for x in h) or (mfe is not None and wf.W(len(c[0])) != mfe):
                bad.append(c)
        finally:
            wf.close()
    print(f"{len(cases)} random folds against the reference driver, {len(bad)} differ")
    assert not bad, bad[:5]
