"""The C++ W_final facade (include/W_final.hh, ccj_amd/csrc/ccj_wfinal.cc) as a drop-in.

oracle/_ref/ccj_ref_main is the reference's OWN unmodified driver — src/CCJ.cc and its gengetopt
parser src/cmdline.cc, compiled from /root/reference by oracle/Makefile (`facade` target) — linked
against libccj_hip.so through our W_final.hh instead of the reference's W_final/pseudo_loop.  It
must behave exactly like the stock reference binary (tests/golden/cli.json, recorded from
oracle/_ref/CCJ): option errors, sequence checks and the parameter loader on CPU; the folds on the
GPU.  The binary travels to the GPU box prebuilt (oracle/_ref is not gpurun-ignored).
"""
import os
import subprocess

import pytest

from tests.oracle_lib import ROOT, golden

MAIN = os.path.join(ROOT, "oracle", "_ref", "ccj_ref_main")
G = golden("cli.json")
ARGV0 = G["argv0"]
# the reference's default parameter file is CWD-relative (CCJ.cc:92); the golden scratch
# directory had it, ours does not, so folds without -P are not comparable here
CPU = [c for c in G["cases"] if not c["fold"]]
GPU = [c for c in G["cases"] if c["fold"] and "-P" in c["argv"]]

needs_main = pytest.mark.skipif(not os.path.exists(MAIN), reason="oracle/_ref/ccj_ref_main not built (needs /root/reference)")


def _id(c):
    return " ".join(c["argv"]) or f"stdin={c['stdin'][:12]!r}"


def _run(case, tmp_path):
    for name, text in case["files"].items():
        (tmp_path / name).write_text(text)
    r = subprocess.run([ARGV0] + case["argv"], executable=MAIN, input=case["stdin"], capture_output=True, text=True,
                       cwd=tmp_path, timeout=600)
    return r.returncode, r.stdout, r.stderr


@needs_main
@pytest.mark.parametrize("case", CPU, ids=_id)
def test_reference_driver_on_facade_matches_reference(case, tmp_path):
    assert _run(case, tmp_path) == (case["rc"], case["stdout"], case["stderr"])


@needs_main
def test_reference_driver_exports_its_penalties():
    """The facade reads the program's PK penalty globals (h_globals.hh) through weak references."""
    nm = subprocess.run(["nm", "-D", MAIN], capture_output=True, text=True).stdout
    for sym in ("PS_penalty", "PSM_penalty", "cp_penalty", "e_intP_penalty"):
        assert sym in nm


@needs_main
@pytest.mark.gpu
@pytest.mark.parametrize("case", GPU, ids=_id)
def test_reference_driver_on_facade_folds_like_reference(case, tmp_path):
    assert _run(case, tmp_path) == (case["rc"], case["stdout"], case["stderr"])


@needs_main
@pytest.mark.gpu
def test_ref_compat_abort_reproduces_stock_n214_abort(tmp_path):
    """CCJ_REF_COMPAT_ABORT=1: the stock build's assert (matrices.hh:160) for n >= 214, before any
    output; n = 213 still folds."""
    import random
    r = random.Random(1)
    seq = "".join(r.choice("ACGU") for _ in range(214))
    par = [c for c in G["cases"] if c["files"] and c["fold"] and c["rc"] == 0][0]
    name, text = next(iter(par["files"].items()))
    (tmp_path / name).write_text(text)
    env = dict(os.environ, CCJ_REF_COMPAT_ABORT="1")
    p = subprocess.run([ARGV0, "-P", name, seq], executable=MAIN, capture_output=True, text=True, cwd=tmp_path,
                       env=env, timeout=600)
    assert p.returncode == -6 and p.stdout == ""
    assert "Assertion `slice_size_ == n*(n+1)*(n+2)*(n+3)/24' failed." in p.stderr
