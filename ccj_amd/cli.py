"""CCJ command line, mirroring the reference driver (src/CCJ.cc:58-115, src/ccj.ggo:1-33).

    CCJ [-i FILE] [-d N] [-P paramfile] [--noConv] [--noGU] [sequence]

Behaviour kept from the reference:
  * the sequence comes from the first positional argument, else the first stdin line — unless
    -i is given, in which case it is NOT read at all (CCJ.cc:68-72: -i is parsed but ignored),
  * upper-casing, T->U unless --noConv, validation messages on stdout with exit code 1,
  * a 'T' left in the sequence (only with --noConv) selects DNA Mathews 2004 and forces noGU,
  * "Not a valid parameter file!" on stderr with exit code 1 for a missing -P file,
  * stdout: optional "Should not be here!" lines, then SEQ, then "STRUCT (E)" with E printed like
    std::cout (6 significant digits, %g), reference backtrack exits reproduced (stderr + code).
Deliberate difference: without -P the reference reads params/rna_DirksPierce09.par relative to
the current directory (CCJ.cc:92) and fails elsewhere; here the DirksPierce09 tables always load.
-P accepts one of our table blobs (*.ccjp) or a reference parameter file name (rna_Turner04.par
...), which selects the matching blob.
"""
from __future__ import annotations

import argparse
import os
import sys

from . import BacktrackExit, CCJError, W_final, param_path


def fmt_energy(e: float) -> str:
    """std::ostream default formatting of a double (precision 6, like %g)."""
    return "%g" % e


def run(argv=None, stdin=None, stdout=None, stderr=None) -> int:
    stdin = stdin or sys.stdin
    stdout = stdout or sys.stdout
    stderr = stderr or sys.stderr
    ap = argparse.ArgumentParser(prog="CCJ", description="Read RNA sequence from stdin or cmdline; predict "
                                 "minimum free energy and optimum structure")
    ap.add_argument("-i", "--input-file", dest="input_file")
    ap.add_argument("-d", "--dangles", type=int, default=2)
    ap.add_argument("-P", "--paramFile", dest="param_file")
    ap.add_argument("--noConv", action="store_true")
    ap.add_argument("--noGU", action="store_true")
    ap.add_argument("--device", type=int, default=int(os.environ.get("LOCAL_RANK", "0")))
    ap.add_argument("inputs", nargs="*")
    a = ap.parse_args(argv)

    seq = ""
    if a.inputs:
        seq = a.inputs[0]
    elif a.input_file is None:
        seq = stdin.readline().rstrip("\n")
    seq = seq.upper()
    if not a.noConv:
        seq = seq.replace("T", "U")
    noGU = a.noGU
    if len(seq) == 0:
        print("sequence is missing", file=stdout)
        return 1
    for c in seq:
        if c not in "GCAUT":
            print(f"Sequence contains character {c} that is not G,C,A,U, or T.", file=stdout)
            return 1
    if a.param_file is not None:
        if not os.path.exists(a.param_file):
            print("Not a valid parameter file!", file=stderr)
            return 1
        try:
            params = param_path(a.param_file)
        except CCJError as e:
            print(f"unsupported parameter file (only the reference's sets are tabulated): {e.msg}", file=stderr)
            return 1
    elif "T" in seq:
        noGU = True
        params = "DNA_Mathews2004"
    else:
        params = "DirksPierce09"
    code, out, err = fold_cli(seq, params, a.dangles, noGU, device=a.device)
    stdout.write(out)
    stderr.write(err)
    stdout.flush()
    return code


def fold_cli(seq: str, params: str, dangles: int, noGU: bool, device: int = 0):
    """One CCJ invocation -> (exit code, stdout text, stderr text), as the reference prints them."""
    wf = W_final(seq, dangles, params=params, noGU=noGU, device=device)
    try:
        energy = wf.ccj()
    except BacktrackExit as e:
        return e.exit_code, e.stdout, e.msg
    finally:
        msgs = wf.stdout_msgs
        wf.close()
    return 0, msgs + seq + "\n" + f"{wf.structure} ({fmt_energy(energy)})\n", ""


def main():
    sys.exit(run())
