"""ctypes binding of the C restatement (oracle/ccj_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module; the
engine never does.  If oracle/_ref/libccj_oracle.so is absent it is compiled with gcc.
"""
import ctypes
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_ref", "libccj_oracle.so")
REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
GOLDEN = os.path.join(ROOT, "tests", "golden")
HASH_NAMES = ["PK", "PL", "PR", "PM", "PO", "PfromL", "PfromR", "PfromM", "PfromMprime", "PfromO",
              "PLmloop00", "PLmloop01", "PLmloop10", "PRmloop00", "PRmloop01", "PRmloop10",
              "PMmloop00", "PMmloop01", "PMmloop10", "POmloop00", "POmloop01", "POmloop10",
              "P", "WBP", "WPP", "V", "Vtype", "WM", "WMv", "WMp", "W"]

_lib = None


def oracle_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True,
                           capture_output=True)
        L = ctypes.CDLL(ORACLE_SO)
        L.ccj_oracle_fold.restype = ctypes.c_void_p
        L.ccj_oracle_fold.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.ccj_oracle_fold_par.restype = ctypes.c_void_p
        L.ccj_oracle_fold_par.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ccj_oracle_hashes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        L.ccj_oracle_free.argtypes = [ctypes.c_void_p]
        L.ccj_oracle_W.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ccj_oracle_get4.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5
        L.ccj_oracle_get4.restype = ctypes.c_int
        L.ccj_oracle_get2.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 3
        L.ccj_oracle_get2.restype = ctypes.c_int
        L.ccj_oracle_W.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ccj_oracle_W.restype = ctypes.c_int
        _lib = L
    return _lib


class OracleFold:
    """CPU restatement of the fill for one sequence (reference loop order)."""

    def __init__(self, seq, blob: bytes, dangles=2, noGU=0, threads=None):
        """threads=None: the sequential fill in the reference's own loop order; threads=k (0: all
        cores): the level-parallel restatement (ccj_oracle_fold_par, OpenMP)."""
        L = oracle_lib()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        self.n = len(seq)
        if threads is None:
            self.h = L.ccj_oracle_fold(seq.encode(), self._blob, dangles, noGU)
        else:
            self.h = L.ccj_oracle_fold_par(seq.encode(), self._blob, dangles, noGU, threads)
        if not self.h:
            raise MemoryError("oracle allocation failed")

    def hashes(self):
        out = (ctypes.c_uint64 * 31)()
        oracle_lib().ccj_oracle_hashes(self.h, out)
        return {HASH_NAMES[i]: "%016x" % out[i] for i in range(31)}

    def get4(self, m, i, j, k, l):
        return oracle_lib().ccj_oracle_get4(self.h, m, i, j, k, l)

    def get2(self, m, i, j):
        return oracle_lib().ccj_oracle_get2(self.h, m, i, j)

    def W(self, j):
        return oracle_lib().ccj_oracle_W(self.h, j)

    def close(self):
        if self.h:
            oracle_lib().ccj_oracle_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def blob(name):
    with open(os.path.join(ROOT, "ccj_amd", "params", name + ".ccjp"), "rb") as f:
        return f.read()
