"""The CCJ command line against the reference CLI (tests/golden/cli.json, made by
oracle/gen_cli_golden.py from oracle/_ref/CCJ): help/version text, every option-parser error,
sequence validation, -P handling (missing file, native .par warnings and fatal errors), exit
codes — for both the native binary ccj_amd/bin/CCJ and the Python CLI ccj_amd.cli.
Cases that stop before the fill run on CPU; the ones that fold are @gpu."""
import io
import os
import subprocess

import pytest

from tests.oracle_lib import ROOT, golden

BIN = os.path.join(ROOT, "ccj_amd", "bin", "CCJ")
G = golden("cli.json")
ARGV0 = G["argv0"]
CPU = [c for c in G["cases"] if not c["fold"]]
GPU = [c for c in G["cases"] if c["fold"]]


def _id(c):
    return " ".join(c["argv"]) or f"stdin={c['stdin'][:12]!r}"


def _run_binary(case, tmp_path):
    for name, text in case["files"].items():
        (tmp_path / name).write_text(text)
    env = dict(os.environ)
    r = subprocess.run([ARGV0] + case["argv"], executable=BIN, input=case["stdin"], capture_output=True, text=True,
                       cwd=tmp_path, env=env, timeout=600)
    return r.returncode, r.stdout, r.stderr


def _run_python(case, tmp_path, monkeypatch):
    from ccj_amd.cli import run
    for name, text in case["files"].items():
        (tmp_path / name).write_text(text)
    monkeypatch.chdir(tmp_path)
    out, err = io.StringIO(), io.StringIO()
    rc = run(case["argv"], stdin=io.StringIO(case["stdin"]), stdout=out, stderr=err, prog=ARGV0)
    return rc, out.getvalue(), err.getvalue()


def _expect(case):
    return case["rc"], case["stdout"], case["stderr"]


@pytest.mark.parametrize("case", CPU, ids=_id)
def test_binary_cli_matches_reference(case, tmp_path):
    assert os.path.exists(BIN), "run __graft_entry__.build() first"
    assert _run_binary(case, tmp_path) == _expect(case)


@pytest.mark.parametrize("case", CPU, ids=_id)
def test_python_cli_matches_reference(case, tmp_path, monkeypatch):
    assert _run_python(case, tmp_path, monkeypatch) == _expect(case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", GPU, ids=_id)
def test_binary_cli_folds_like_reference(case, tmp_path):
    assert _run_binary(case, tmp_path) == _expect(case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", GPU, ids=_id)
def test_python_cli_folds_like_reference(case, tmp_path, monkeypatch):
    assert _run_python(case, tmp_path, monkeypatch) == _expect(case)
