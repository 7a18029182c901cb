"""CCJ command line, mirroring the reference driver (src/CCJ.cc:58-115) and its gengetopt parser
(src/ccj.ggo:1-33, src/cmdline.cc:375-640).

    CCJ [-h] [-V] [-i FILE] [-d N] [-P paramfile] [--noConv] [--noGU] [sequence]

Same behaviour as ccj_amd/bin/CCJ (ccj_amd/csrc/ccj_cli.cc):
  * options parsed like glibc getopt_long over the reference's table: argument permutation,
    "--" terminator, unique-prefix long options ("--no" = --noConv: both candidates share
    has_arg/flag/val so glibc takes the first), clustered short options, glibc's messages with
    argv[0]; -h / -V print and exit 0 when reached; repeated options and bad -d values fail with
    gengetopt's messages (exit 1); -d is strtol(base 0), e.g. "0x2" is 2;
  * the sequence comes from the first non-option argument, else the first stdin line — unless
    -i is given, in which case it is NOT read at all (CCJ.cc:68-72: -i is parsed but ignored);
  * upper-casing, T->U unless --noConv, validation messages on stdout with exit code 1,
  * a 'T' left in the sequence (only with --noConv) selects DNA Mathews 2004 and forces noGU,
  * "Not a valid parameter file!" on stderr with exit code 1 for a missing -P path; any other
    -P file is read natively as a ViennaRNA v2.0 .par file (warnings/errors as the reference
    prints them; a fatal one exits 1), a *.ccjp path is one of our table blobs;
  * stdout: optional "Should not be here!" lines, then SEQ, then "STRUCT (E)" with E printed like
    std::cout (6 significant digits, %g), reference backtrack exits reproduced (stderr + code).
Without -P the reference reads params/rna_DirksPierce09.par relative to the current directory
(CCJ.cc:92); that file is read when present, otherwise the bundled DirksPierce09 tables are used
where the reference would fail.  Device: $CCJ_DEVICE, else $LOCAL_RANK, else 0.
"""
from __future__ import annotations

import os
import sys

from . import BacktrackExit, ParFileError, W_final, load_par

HELP = """Usage: CCJ [options] [sequence]
Pseudoknotted minimum free energy folding of RNAs

Read RNA sequence from stdin or cmdline; predict minimum
free energy and optimum structure

  -h, --help               Print help and exit
  -V, --version            Print version and exit
  -i, --input-file=STRING  Give a path to an input file containing the sequence
                             (and input structure if known)
  -d, --dangles=INT        Specify the dangle model to be used (base is 2)
                             (default=`2')
  -P, --paramFile=STRING   Read energy parameters from paramfile, instead of
                             using the default parameter set.
      --noConv             Do not convert DNA into RNA. This will use the
                             Matthews 2004 parameters for DNA  (default=off)
      --noGU               Turn off G-U and U-G (and G-T and T-G) base pairing
                             (default=off)

The input sequence is read from standard input, unless it is
given on the command line.

"""
VERSION = "CCJ 1.0\n"
# vrna_params_load_DNA_Mathews2004() runs check_symmetry (io.c:1126) over the built-in DNA set,
# whose stack enthalpies are asymmetric in two pairs: the reference prints this on every DNA run.
DNA_WARNINGS = "WARNING: stacking enthalpies not symmetric\n" * 4

# (name, takes_argument, short letter or None) — reference cmdline.cc:511-520
LONG_OPTS = [("help", False, "h"), ("version", False, "V"), ("input-file", True, "i"), ("dangles", True, "d"),
             ("paramFile", True, "P"), ("noConv", False, None), ("noGU", False, None)]
SHORT_OPTS = {"h": False, "V": False, "i": True, "d": True, "P": True}


class _Stop(Exception):
    def __init__(self, code, out="", err=""):
        self.code, self.out, self.err = code, out, err


def getopt_long(argv):
    """glibc getopt_long (permuting) over the reference table.  Yields (name, arg) in the order
    options appear; returns the non-option arguments at the end via StopIteration.value.
    Raises _Stop(1, err=message) where getopt prints an error."""
    prog = argv[0]
    rest, k = [], 1
    while k < len(argv):
        a = argv[k]
        k += 1
        if a == "--":
            rest.extend(argv[k:])
            break
        if not a.startswith("-") or a == "-":
            rest.append(a)
            continue
        if a.startswith("--"):
            body = a[2:]
            name, eq, val = body.partition("=")
            exact = [o for o in LONG_OPTS if o[0] == name]
            cands = exact or [o for o in LONG_OPTS if o[0].startswith(name)]
            if not cands:
                raise _Stop(1, err=f"{prog}: unrecognized option '--{body}'\n")
            opt = cands[0]
            # glibc: a prefix match is ambiguous when a later candidate differs from the first in
            # has_arg/flag/val (noConv and noGU do not differ: both are {0, NULL, 0})
            ambig = [o for o in cands[1:] if o[1] != opt[1] or (o[2] or "") != (opt[2] or "")]
            if ambig:
                names = " ".join(f"'--{o[0]}'" for o in [opt] + ambig)
                raise _Stop(1, err=f"{prog}: option '--{body}' is ambiguous; possibilities: {names}\n")
            if opt[1]:
                if not eq:
                    if k >= len(argv):
                        raise _Stop(1, err=f"{prog}: option '--{opt[0]}' requires an argument\n")
                    val = argv[k]
                    k += 1
                yield opt[0], val
            else:
                if eq:
                    raise _Stop(1, err=f"{prog}: option '--{opt[0]}' doesn't allow an argument\n")
                yield opt[0], None
            continue
        j = 1
        while j < len(a):
            ch = a[j]
            j += 1
            if ch not in SHORT_OPTS:
                raise _Stop(1, err=f"{prog}: invalid option -- '{ch}'\n")
            long_name = next(o[0] for o in LONG_OPTS if o[2] == ch)
            if SHORT_OPTS[ch]:
                if j < len(a):
                    val = a[j:]
                elif k < len(argv):
                    val = argv[k]
                    k += 1
                else:
                    raise _Stop(1, err=f"{prog}: option requires an argument -- '{ch}'\n")
                yield long_name, val
                break
            yield long_name, None
    return rest


def _strtol0(s: str):
    """C strtol(s, &end, 0) -> (value, fully_consumed)."""
    t = s.lstrip(" \t\n\v\f\r")
    sign, i = 1, 0
    if t[:1] in "+-" and t:
        sign = -1 if t[0] == "-" else 1
        i = 1
    base, digits = 10, "0123456789"
    if t[i:i + 2].lower() == "0x" and len(t) > i + 2 and t[i + 2].lower() in "0123456789abcdef":
        base, i, digits = 16, i + 2, "0123456789abcdef"
    elif t[i:i + 1] == "0":
        base, digits = 8, "01234567"
    j = i
    while j < len(t) and t[j].lower() in digits:
        j += 1
    if j == i:
        return 0, s == ""  # no conversion: end pointer = start, so only "" passes gengetopt's check
    v = sign * int(t[i:j], base)
    v = max(-2**63, min(2**63 - 1, v))  # long saturation
    v = (v + 2**31) % 2**32 - 2**31  # stored into an int
    return v, j == len(t)


def parse(argv):
    """gengetopt cmdline_parser -> dict of option values (reference cmdline.cc:490-640)."""
    prog = argv[0]
    args = {"dangles": 2, "input_file": None, "paramFile": None, "noConv": False, "noGU": False, "inputs": []}
    given = {}
    short = {o[0]: o[2] for o in LONG_OPTS}
    gen = getopt_long(argv)
    while True:
        try:
            name, val = next(gen)
        except StopIteration as e:
            args["inputs"] = e.value
            return args
        if name == "help":
            raise _Stop(0, out=HELP)
        if name == "version":
            raise _Stop(0, out=VERSION)
        if given.get(name):
            s = short[name]
            msg = (f"{prog}: `--{name}' (`-{s}') option given more than once\n" if s
                   else f"{prog}: `--{name}' option given more than once\n")
            raise _Stop(1, err=msg)
        given[name] = 1
        if name == "dangles":
            v, ok = _strtol0(val)
            if not ok:
                raise _Stop(1, err=f"{prog}: invalid numeric value: {val}\n")
            args["dangles"] = v
        elif name == "input-file":
            args["input_file"] = val
        elif name == "paramFile":
            args["paramFile"] = val
        else:
            args[name] = True


def fmt_energy(e: float) -> str:
    """std::ostream default formatting of a double (precision 6, like %g)."""
    return "%g" % e


def run(argv=None, stdin=None, stdout=None, stderr=None, prog="CCJ") -> int:
    stdin = stdin or sys.stdin
    stdout = stdout or sys.stdout
    stderr = stderr or sys.stderr
    argv = [prog] + list(sys.argv[1:] if argv is None else argv)
    try:
        a = parse(argv)
        code, out, err = _main(a, stdin)
    except _Stop as s:
        code, out, err = s.code, s.out, s.err
    stdout.write(out)
    stderr.write(err)
    stdout.flush()
    return code


def _main(a, stdin):
    seq = ""
    if a["inputs"]:
        seq = a["inputs"][0]
    elif a["input_file"] is None:
        seq = stdin.readline().rstrip("\n")
    seq = seq.upper()
    if not a["noConv"]:
        seq = seq.replace("T", "U")
    noGU = a["noGU"]
    if len(seq) == 0:
        return 1, "sequence is missing\n", ""
    for c in seq:
        if c not in "GCAUT":
            return 1, f"Sequence contains character {c} that is not G,C,A,U, or T.\n", ""
    err = ""
    if a["paramFile"] is not None:
        pf = a["paramFile"]
        if not os.path.exists(pf):
            return 1, "", "Not a valid parameter file!\n"
        if pf.endswith(".ccjp"):
            params = pf
        else:
            try:
                _, params, err = load_par(pf)
            except ParFileError as e:
                return 1, "", e.log
    elif "T" in seq:
        noGU = True
        params = "DNA_Mathews2004"
        err = DNA_WARNINGS
    elif os.path.exists("params/rna_DirksPierce09.par"):
        try:
            _, params, err = load_par("params/rna_DirksPierce09.par")
        except ParFileError as e:
            return 1, "", e.log
    else:
        params = "DirksPierce09"
    device = int(os.environ.get("CCJ_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    code, out, ferr = fold_cli(seq, params, a["dangles"], noGU, device=device)
    return code, out, err + ferr


def fold_cli(seq: str, params, dangles: int, noGU: bool, device: int = 0):
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
    sys.exit(run(prog=sys.argv[0]))
