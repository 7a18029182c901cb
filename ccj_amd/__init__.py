"""ccj_amd — MI355X-native CCJ pseudoknot MFE engine (host mirror of the reference API).

The reference exposes CCJ through a C++ class and a free function:

    W_final(std::string seq, int dangle);  double W_final::ccj();  std::string W_final::structure
        (reference src/W_final.hh:18-71, src/W_final.cc:20-105)
    std::string ccj(std::string seq, double &energy, int dangle)       (reference src/CCJ.cc:44-49)

This package mirrors that surface in Python on top of libccj_hip.so (include/ccj.h).  The fill
always runs on the GPU through hand-written HIP kernels; there is no CPU fallback — if the
extension is missing or no GPU is visible the calls raise.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

__all__ = [
    "W_final", "ccj", "load_params", "load_par", "ParFileError", "param_path", "CCJError", "BacktrackExit", "lib", "MAT4", "MAT2",
    "num_cells", "comm_unique_id", "shard_blocks", "level_layout", "LocalGroup", "W_final_pf", "PF_MAT4", "PF_MAT2",
    "SampleExit", "pf_exp_hashes", "load_pfraw",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# CCJ_LIB_VARIANT=dbg selects the bounds-checked debug build (libccj_hip_dbg.so); other variants
# (libccj_hip_<name>.so) are timing-only ablation builds made by tools/ablate.sh.
_VARIANT = os.environ.get("CCJ_LIB_VARIANT", "")
_LIB_PATH = os.path.join(_HERE, "lib", f"libccj_hip_{_VARIANT}.so" if _VARIANT else "libccj_hip.so")
PARAM_DIR = os.path.join(_HERE, "params")

# ccj.h enums
MAT4 = ["PK", "PL", "PR", "PM", "PO", "PfromL", "PfromR", "PfromM", "PfromMprime", "PfromO",
        "PLmloop00", "PLmloop01", "PLmloop10", "PRmloop00", "PRmloop01", "PRmloop10",
        "PMmloop00", "PMmloop01", "PMmloop10", "POmloop00", "POmloop01", "POmloop10"]
MAT2 = ["P", "WBP", "WPP", "V", "Vtype", "WM", "WMv", "WMp"]
HASH_NAMES = MAT4 + MAT2 + ["W"]
# ccj_pf.h enums (partition function)
PF_MAT4 = ["PK", "PL", "PR", "PM", "PO", "PfromL", "PfromR", "PfromM", "PfromO",
           "PLmloop00", "PLmloop01", "PLmloop10", "PRmloop00", "PRmloop01", "PRmloop10",
           "PMmloop00", "PMmloop01", "PMmloop10", "POmloop00", "POmloop01", "POmloop10"]
PF_MAT2 = ["V", "VM", "WM", "WMv", "WMp", "WBP", "WPP", "P"]
CCJ_E_PF_SAMPLE = 8  # include/ccj_pf.h

CCJ_OK, CCJ_E_ARG, CCJ_E_OOM, CCJ_E_HIP, CCJ_E_PARAMS, CCJ_E_BACKTRACK, CCJ_E_STATE, CCJ_E_INTER_EXIT = range(8)
CCJ_E_COMM = 9  # include/ccj.h: band-sharded exchange failed or timed out
CCJ_E_PARFILE = 8  # include/ccj_parfile.h

# name -> blob file (the reference's params/*.par sets, dumped to our table format)
PARAM_SETS = {
    "Turner04": "Turner04.ccjp", "rna_Turner04": "Turner04.ccjp",
    "DirksPierce09": "DirksPierce09.ccjp", "rna_DirksPierce09": "DirksPierce09.ccjp",
    "DirksPierce03": "DirksPierce03.ccjp", "rna_DirksPierce03": "DirksPierce03.ccjp",
    "CaoChen06": "CaoChen06.ccjp", "rna_CaoChen06": "CaoChen06.ccjp",
    "CaoChen09": "CaoChen09.ccjp", "rna_CaoChen09": "CaoChen09.ccjp",
    "Matthews04": "Matthews04.ccjp", "dna_Matthews04": "Matthews04.ccjp",
    "DNA_Mathews2004": "DNA_Mathews2004.ccjp", "default": "default.ccjp",
}


class CCJError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ccj error {code}: {msg}")
        self.code = code
        self.msg = msg


class BacktrackExit(CCJError):
    """The reference would have terminated inside its backtrack (stderr text + exit code)."""

    def __init__(self, code: int, msg: str, exit_code: int, stdout: str):
        super().__init__(code, msg)
        self.exit_code = exit_code
        self.stdout = stdout


class _Problem(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_char_p), ("dangles", ctypes.c_int), ("noGU", ctypes.c_int),
                ("params", ctypes.c_void_p), ("pen", ctypes.c_void_p)]


class _Options(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("overlap_d2h", ctypes.c_int), ("shard_world", ctypes.c_int),
                ("shard_rank", ctypes.c_int), ("shard_simulate", ctypes.c_int), ("host_traceback", ctypes.c_int),
                ("split_target", ctypes.c_int), ("share_splits", ctypes.c_int)]

COMM_ID_BYTES = 128


_lib = None


def lib() -> ctypes.CDLL:
    """Load libccj_hip.so (raises if it has not been built — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise CCJError(CCJ_E_STATE, f"{_LIB_PATH} missing: run __graft_entry__.build() first")
    L = ctypes.CDLL(_LIB_PATH)
    vp, ip, cp = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
    L.ccj_create.argtypes = [ctypes.POINTER(_Problem), ctypes.POINTER(_Options), ctypes.POINTER(vp)]
    L.ccj_create.restype = ip
    for fn in ("ccj_fill", "ccj_fill_device", "ccj_sync_host", "ccj_n"):
        getattr(L, fn).argtypes = [vp]
        getattr(L, fn).restype = ip
    L.ccj_reset.argtypes = [vp, cp]
    L.ccj_reset.restype = ip
    L.ccj_fill_async.argtypes = [vp]
    L.ccj_fill_async.restype = ip
    L.ccj_fill_async_after.argtypes = [vp, vp]
    L.ccj_fill_async_after.restype = ip
    L.ccj_wait.argtypes = [vp, cp, ctypes.POINTER(ctypes.c_double), cp, ip]
    L.ccj_wait.restype = ip
    L.ccj_result.argtypes = [vp, cp, ctypes.POINTER(ctypes.c_double), cp, ip]
    L.ccj_result.restype = ip
    L.ccj_get4.argtypes = [vp, ip, ip, ip, ip, ip]
    L.ccj_get4.restype = ip
    L.ccj_get2.argtypes = [vp, ip, ip, ip]
    L.ccj_get2.restype = ip
    L.ccj_getW.argtypes = [vp, ip]
    L.ccj_getW.restype = ip
    L.ccj_hashes.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.ccj_hashes.restype = ip
    L.ccj_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    L.ccj_last_timing.restype = ip
    L.ccj_last_error.argtypes = [vp]
    L.ccj_last_error.restype = cp
    L.ccj_destroy.argtypes = [vp]
    L.ccj_destroy.restype = None
    L.ccj_num_cells.argtypes = [ip]
    L.ccj_num_cells.restype = ctypes.c_uint64
    L.ccj_host_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.ccj_host_timing.restype = ip
    L.ccj_iloop_ms.argtypes = [vp]
    L.ccj_iloop_ms.restype = ctypes.c_double
    L.ccj_ppush_ms.argtypes = [vp]
    L.ccj_ppush_ms.restype = ctypes.c_double
    L.ccj_set_timing.argtypes = [vp, ip]
    L.ccj_set_timing.restype = ip
    L.ccj_comm_unique_id.argtypes = [cp]
    L.ccj_comm_unique_id.restype = ip
    L.ccj_comm_init.argtypes = [vp, cp]
    L.ccj_comm_init.restype = ip
    L.ccj_shard_blocks.argtypes = [ip, ip, ip, ip, ctypes.POINTER(ip), ip]
    L.ccj_shard_blocks.restype = ip
    L.ccj_group_create.argtypes = [ip, ctypes.POINTER(vp)]
    L.ccj_group_create.restype = ip
    L.ccj_group_destroy.argtypes = [vp]
    L.ccj_group_destroy.restype = None
    L.ccj_comm_init_local.argtypes = [vp, vp]
    L.ccj_comm_init_local.restype = ip
    L.ccj_level_layout.argtypes = [ip, ip, ip, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ip)]
    L.ccj_level_layout.restype = ip
    L.ccj_params_load_par.argtypes = [cp, cp, cp, cp, ip]
    L.ccj_params_load_par.restype = ip
    L.ccj_params_load_par_string.argtypes = [cp, cp, cp, cp, ip]
    L.ccj_params_load_par_string.restype = ip
    # partition function (include/ccj_pf.h)
    u64p, dp = ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)
    L.ccj_pf_create.argtypes = [ctypes.POINTER(_Problem), cp, ip, ctypes.POINTER(vp)]
    L.ccj_pf_create.restype = ip
    L.ccj_pf_destroy.argtypes = [vp]
    L.ccj_pf_destroy.restype = None
    L.ccj_pf_fill.argtypes = [vp, dp]
    L.ccj_pf_fill.restype = ip
    L.ccj_pf_W.argtypes = [vp, dp]
    L.ccj_pf_W.restype = ip
    L.ccj_pf_get2.argtypes = [vp, ip, dp]
    L.ccj_pf_get2.restype = ip
    L.ccj_pf_get4.argtypes = [vp, ip, ip, ip, ip, ip, ctypes.POINTER(ip)]
    L.ccj_pf_get4.restype = ip
    L.ccj_pf_hashes.argtypes = [vp, u64p, u64p]
    L.ccj_pf_hashes.restype = ip
    L.ccj_pf_exp_hashes.argtypes = [vp, u64p, ip]
    L.ccj_pf_exp_hashes.restype = ip
    L.ccj_pf_exp_hashes_params.argtypes = [cp, cp, vp, u64p, ip]
    L.ccj_pf_exp_hashes_params.restype = ip
    L.ccj_pf_exp_names.argtypes = []
    L.ccj_pf_exp_names.restype = cp
    L.ccj_pf_srand.argtypes = [vp, ctypes.c_uint]
    L.ccj_pf_srand.restype = ip
    L.ccj_pf_sample.argtypes = [vp, ip, cp, ctypes.POINTER(ip)]
    L.ccj_pf_sample.restype = ip
    L.ccj_pf_last_message.argtypes = [vp]
    L.ccj_pf_last_message.restype = cp
    L.ccj_pf_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.ccj_pf_timing.restype = ip
    L.ccj_pf_set_timing.argtypes = [vp, ip]
    L.ccj_pf_set_timing.restype = ip
    L.ccj_pf_kernel_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.ccj_pf_kernel_ms.restype = ip
    L.ccj_pf_work_model.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.ccj_pf_work_model.restype = ip
    _lib = L
    return L


def num_cells(n: int) -> int:
    """4-D DP cells C(n+1,4) — the unit of work."""
    if n < 3:
        return 0
    m = n + 1
    return m * (m - 1) * (m - 2) * (m - 3) // 24


def param_path(name_or_path: str) -> str:
    """Bundled blob for a parameter-set name ("Turner04", "rna_Turner04.par", ...) or a .ccjp path."""
    if os.path.exists(name_or_path) and name_or_path.endswith(".ccjp"):
        return name_or_path
    base = os.path.basename(name_or_path)
    for suf in (".par", ".ccjp"):
        if base.endswith(suf):
            base = base[: -len(suf)]
    if base in PARAM_SETS:
        return os.path.join(PARAM_DIR, PARAM_SETS[base])
    raise CCJError(CCJ_E_ARG, f"unknown parameter set {name_or_path!r}")


class ParFileError(CCJError):
    """A .par file the reference loader rejects: it prints ``log`` on stderr and exits 1."""

    def __init__(self, log: str):
        super().__init__(CCJ_E_PARFILE, log)
        self.log = log


def load_par(path: str, base: bytes | None = None, text: bool = False):
    """Read a ViennaRNA v2.0 parameter file natively (include/ccj_parfile.h).

    ``base`` is the table state the file lands on (default: the reference's compiled-in
    defaults, ccj_amd/params/default.ccjp).  ``text=True`` treats ``path`` as the file contents
    (vrna_params_load_from_string).  Returns (applied, blob, log): applied is 1 when the file was
    parsed, 0 when it could not be opened or was empty (blob == base); log is what the reference
    prints on stderr.  Raises ParFileError where the reference exits 1.
    """
    if base is None:
        base = _read_blob(os.path.join(PARAM_DIR, "default.ccjp"))
    L = lib()
    out = ctypes.create_string_buffer(len(base))
    cap = 1 << 22
    log = ctypes.create_string_buffer(cap)
    fn = L.ccj_params_load_par_string if text else L.ccj_params_load_par
    rc = fn(path.encode(), bytes(base), out, log, cap)
    msg = log.value.decode(errors="replace")
    if rc == CCJ_E_PARFILE:
        raise ParFileError(msg)
    if rc < 0:
        raise CCJError(CCJ_E_ARG, "bad parameter base blob")
    return rc, out.raw, msg


def _read_blob(p: str) -> bytes:
    if p not in _PARAM_CACHE:
        with open(p, "rb") as f:
            _PARAM_CACHE[p] = f.read()
    return _PARAM_CACHE[p]


_PARAM_CACHE: dict = {}


def load_params(name_or_path: str = "DirksPierce09") -> bytes:
    """Scaled 37 C energy tables (include/ccj_params.h).

    An existing .par file is read natively over the compiled-in defaults (like the reference's
    vrna_params_load); an existing .ccjp is used as is; otherwise the name selects one of the
    bundled sets (Turner04, DirksPierce09, ... — dumps of the reference's own files).
    """
    if os.path.isfile(name_or_path) and not name_or_path.endswith(".ccjp"):
        key = ("par", os.path.abspath(name_or_path), os.path.getmtime(name_or_path))
        if key not in _PARAM_CACHE:
            _PARAM_CACHE[key] = load_par(name_or_path)[1]
        return _PARAM_CACHE[key]
    return _read_blob(param_path(name_or_path))


class W_final:
    """Mirror of the reference class W_final (src/W_final.hh:18-71).

    ``W_final(seq, dangle).ccj()`` fills every matrix on the GPU, runs W + backtrack on the host
    mirror and returns the MFE in kcal/mol; ``structure`` holds the dot-bracket string.
    """

    def __init__(self, seq: str, dangle: int = 2, params: str | bytes = "DirksPierce09",
                 noGU: bool = False, device: int = 0, overlap_d2h: bool = False, shard_world: int = 1,
                 shard_rank: int = 0, shard_simulate: bool = False, comm_id: Optional[bytes] = None,
                 host_traceback: bool = False, split_target: int = 0, share_splits: int = 0,
                 local_group: Optional["LocalGroup"] = None):
        """shard_world > 1: band-shard this one sequence over shard_world processes (one per GPU),
        exchanging each level over RCCL; every rank passes the same comm_id (from comm_unique_id()
        on one rank), or the same local_group when the ranks are contexts of this process.
        shard_simulate runs all shards in this one context without an exchange.
        host_traceback: run W and the traceback on the host over a mirror of every matrix (the
        reference restatement; overlap_d2h streams that mirror during the fill) instead of on the GPU.
        split_target / share_splits: level-kernel tuning (include/ccj.h ccj_options; 0 = default,
        < 0 = never split a level / no split-point sharing)."""
        self.seq = seq
        self.n = len(seq)
        self.dangle = dangle
        self._blob = params if isinstance(params, (bytes, bytearray)) else load_params(params)
        self._blob_buf = ctypes.create_string_buffer(bytes(self._blob), len(self._blob))
        self._seq_buf = ctypes.create_string_buffer(seq.encode())
        L = lib()
        prob = _Problem(ctypes.cast(self._seq_buf, ctypes.c_char_p), dangle, 1 if noGU else 0,
                        ctypes.cast(self._blob_buf, ctypes.c_void_p), None)
        opts = _Options(device, 1 if overlap_d2h else 0, shard_world, shard_rank, 1 if shard_simulate else 0,
                        1 if host_traceback else 0, split_target, share_splits)
        h = ctypes.c_void_p()
        rc = L.ccj_create(ctypes.byref(prob), ctypes.byref(opts), ctypes.byref(h))
        if rc != CCJ_OK:
            raise CCJError(rc, L.ccj_last_error(None).decode())
        self._h = h
        if shard_world > 1 and not shard_simulate and local_group is not None:
            self._group = local_group  # keeps the group alive as long as this context
            self._check(L.ccj_comm_init_local(h, local_group._h))
        elif shard_world > 1 and not shard_simulate:
            if comm_id is None or len(comm_id) != COMM_ID_BYTES:
                raise CCJError(CCJ_E_ARG, "sharded context needs the 128-byte comm_id of rank 0")
            self._check(L.ccj_comm_init(h, comm_id))
        self.structure: Optional[str] = None
        self.energy: Optional[float] = None
        self.stdout_msgs = ""

    def reset(self, seq: str) -> None:
        """Rebind this context to another sequence of the same length (include/ccj.h ccj_reset):
        the allocations are reused, only the sequence tables and work lists are rebuilt."""
        if len(seq) != self.n:
            raise CCJError(CCJ_E_ARG, f"reset: length {len(seq)} differs from n={self.n}")
        self._check(lib().ccj_reset(self._h, seq.encode()))
        self.seq = seq
        self._seq_buf = ctypes.create_string_buffer(seq.encode())
        self.structure = None
        self.energy = None
        self.stdout_msgs = ""

    def _check(self, rc: int):
        if rc != CCJ_OK:
            raise CCJError(rc, lib().ccj_last_error(self._h).decode())

    def fill(self):
        self._check(lib().ccj_fill(self._h))

    def fill_device(self):
        self._check(lib().ccj_fill_device(self._h))

    def sync_host(self):
        self._check(lib().ccj_sync_host(self._h))

    def result(self):
        L = lib()
        buf = ctypes.create_string_buffer(self.n + 1)
        msgs = ctypes.create_string_buffer(1 << 16)
        e = ctypes.c_double()
        rc = L.ccj_result(self._h, buf, ctypes.byref(e), msgs, 1 << 16)
        self.stdout_msgs = msgs.value.decode()
        if rc == CCJ_E_BACKTRACK or rc == CCJ_E_INTER_EXIT:
            err = L.ccj_last_error(self._h).decode()
            exit_code = 0 if rc == CCJ_E_INTER_EXIT else (134 if "Assertion" in err else 1)
            raise BacktrackExit(rc, err, exit_code, self.stdout_msgs)
        self._check(rc)
        self.structure = buf.value.decode()
        self.energy = e.value
        return self.energy

    def ccj(self) -> float:
        """reference W_final::ccj (W_final.cc:58-105)"""
        self.fill()
        return self.result()

    def fill_async(self, after: Optional["W_final"] = None) -> None:
        """Enqueue fill + W + traceback and return at once (include/ccj.h ccj_fill_async); with
        `after`, the fill starts when that context's last enqueued fill has ended."""
        if after is None:
            self._check(lib().ccj_fill_async(self._h))
        else:
            self._check(lib().ccj_fill_async_after(self._h, after._h))

    def wait(self) -> float:
        """Finish a fill_async: same results (and exceptions) as ccj()."""
        L = lib()
        buf = ctypes.create_string_buffer(self.n + 1)
        msgs = ctypes.create_string_buffer(1 << 16)
        e = ctypes.c_double()
        rc = L.ccj_wait(self._h, buf, ctypes.byref(e), msgs, 1 << 16)
        self.stdout_msgs = msgs.value.decode()
        if rc == CCJ_E_BACKTRACK or rc == CCJ_E_INTER_EXIT:
            err = L.ccj_last_error(self._h).decode()
            exit_code = 0 if rc == CCJ_E_INTER_EXIT else (134 if "Assertion" in err else 1)
            raise BacktrackExit(rc, err, exit_code, self.stdout_msgs)
        self._check(rc)
        self.structure = buf.value.decode()
        self.energy = e.value
        return self.energy

    # ---- matrix access (reference getter semantics) ----
    def get4(self, mat, i, j, k, l) -> int:
        m = MAT4.index(mat) if isinstance(mat, str) else mat
        return lib().ccj_get4(self._h, m, i, j, k, l)

    def get2(self, mat, i, j) -> int:
        m = MAT2.index(mat) if isinstance(mat, str) else mat
        return lib().ccj_get2(self._h, m, i, j)

    def W(self, j) -> int:
        return lib().ccj_getW(self._h, j)

    def hashes(self) -> dict:
        out = (ctypes.c_uint64 * len(HASH_NAMES))()
        self._check(lib().ccj_hashes(self._h, out))
        return {name: "%016x" % out[x] for x, name in enumerate(HASH_NAMES)}

    def set_timing(self, mode: int) -> None:
        """What later ccj() calls time: 0 = the fill; 1 (default) = + level durations; 2 = + per-kernel
        family times (k_diag2d, k_iloop) from extra marker events, which slow the fill down."""
        self._check(lib().ccj_set_timing(self._h, mode))

    def timing(self) -> dict:
        f = ctypes.c_double()
        k = (ctypes.c_double * 3)()
        lib().ccj_last_timing(self._h, ctypes.byref(f), k)
        hst = (ctypes.c_double * 3)()
        lib().ccj_host_timing(self._h, hst)
        L = lib()
        return {"fill_ms": f.value, "level4d_ms": k[0], "iloop_ms": L.ccj_iloop_ms(self._h), "diag2d_ms": k[1],
                "ppush_ms": L.ccj_ppush_ms(self._h),
                "precompute_ms": k[2],
                "host_mirror_wait_ms": hst[0], "W_ms": hst[1], "backtrack_ms": hst[2]}

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().ccj_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id for a sharded fold (broadcast it to every rank)."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    rc = lib().ccj_comm_unique_id(buf)
    if rc != CCJ_OK:
        raise CCJError(rc, "ncclGetUniqueId failed")
    return buf.raw


def shard_blocks(n: int, t: int, world: int, rank: int):
    """a-blocks of 4-D level t that rank computes in a band-sharded fold, ascending (no GPU needed):
    block a belongs to rank (a // 4) % world on every level."""
    cap = t + 1
    buf = (ctypes.c_int * max(cap, 1))()
    cnt = lib().ccj_shard_blocks(n, t, world, rank, buf, cap)
    if cnt < 0:
        raise CCJError(-cnt, "bad shard arguments")
    return list(buf[:cnt])


class LocalGroup:
    """In-process exchange group for a band-sharded fold whose ranks are contexts of this process
    (include/ccj.h ccj_group): pass it as W_final(..., shard_world=N, shard_rank=r, local_group=g)
    and drive each rank's fill from its own thread."""

    def __init__(self, world: int):
        h = ctypes.c_void_p()
        rc = lib().ccj_group_create(world, ctypes.byref(h))
        if rc != CCJ_OK:
            raise CCJError(rc, "ccj_group_create failed")
        self._h = h
        self.world = world

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().ccj_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def level_layout(n: int, t: int, world: int):
    """(C_t, M_t): per-matrix element stride of level t (padded to world equal chunks), a-block size."""
    C, M = ctypes.c_longlong(), ctypes.c_int()
    rc = lib().ccj_level_layout(n, t, world, ctypes.byref(C), ctypes.byref(M))
    if rc != CCJ_OK:
        raise CCJError(rc, "bad layout arguments")
    return C.value, M.value


def ccj(seq: str, dangle: int = 2, params: str | bytes = "DirksPierce09", noGU: bool = False,
        device: int = 0):
    """reference ``std::string ccj(std::string seq, double &energy, int dangle)`` (CCJ.cc:44-49).

    Returns (structure, energy_kcal_per_mol).
    """
    wf = W_final(seq, dangle, params=params, noGU=noGU, device=device)
    try:
        energy = wf.ccj()
        return wf.structure, energy
    finally:
        wf.close()


def load_pfraw(name_or_path) -> Optional[bytes]:
    """Raw (unclamped) dangle / mismatch tables of a bundled set (ccj_amd/params/<set>.pfraw,
    include/ccj_pf.h ccj_pf_raw), or None (the engine then takes the pair-type-0 rows as INF)."""
    if not isinstance(name_or_path, str):
        return None
    if os.path.isfile(name_or_path) and not name_or_path.endswith(".ccjp"):
        return None  # a .par file read natively: no raw tables (type-0 rows taken as INF)
    try:
        p = param_path(name_or_path)
    except Exception:
        return None
    raw = p[:-5] + ".pfraw" if p.endswith(".ccjp") else None
    if raw and os.path.exists(raw):
        return _read_blob(raw)
    return None


def pf_exp_hashes(params: str | bytes = "DirksPierce09") -> dict:
    """FNV-1a of the partition function's Boltzmann tables for a parameter set (host only)."""
    blob = params if isinstance(params, (bytes, bytearray)) else load_params(params)
    raw = load_pfraw(params)
    names = lib().ccj_pf_exp_names().decode().split()
    out = (ctypes.c_uint64 * len(names))()
    got = lib().ccj_pf_exp_hashes_params(bytes(blob), raw, None, out, len(names))
    if got != len(names):
        raise CCJError(CCJ_E_ARG, "ccj_pf_exp_hashes_params")
    return {k: "%016x" % v for k, v in zip(names, out)}


class SampleExit(CCJError):
    """A Sample_* failure path of the reference (it prints ``stdout`` and calls exit(0))."""

    def __init__(self, msg: str, structures: list):
        super().__init__(CCJ_E_PF_SAMPLE, msg)
        self.stdout = msg
        self.structures = structures


class W_final_pf:
    """Mirror of the reference class W_final_pf (src/part_func.hh:28-194, part_func.cc).

    ``W_final_pf(seq, MFE_structure, MFE_energy, dangle, num_samples, PSplot).ccj_pf()`` runs the
    CCJ partition function on the GPU (include/ccj_pf.h) and returns the ensemble free energy in
    kcal/mol, bit-identical to the reference's part_func.cc evaluated without floating-point
    contraction.  MFE_structure, MFE_energy and PSplot are accepted and stored like the reference
    (which ignores them: pf_scale is forced to 1).  ``srand(seed)`` + ``sample(k)`` is the
    reference's stochastic traceback Sample_W(1, n) (stoch_backtrack.cc), drawing rand()/RAND_MAX
    like vrna_urn() in the reference build.
    """

    def __init__(self, seq: str, MFE_structure: str = "", MFE_energy: float = 0.0, dangle: int = 2,
                 num_samples: int = 0, PSplot: bool = False, params: str | bytes = "DirksPierce09",
                 noGU: bool = False, device: int = 0):
        self.seq = seq
        self.n = len(seq)
        self.MFE_structure = MFE_structure
        self.MFE_energy = MFE_energy
        self.num_samples = num_samples
        self.PSplot = PSplot
        self.structure = "." * self.n
        self.structures: dict = {}
        self._blob = params if isinstance(params, (bytes, bytearray)) else load_params(params)
        self._blob_buf = ctypes.create_string_buffer(bytes(self._blob), len(self._blob))
        self._seq_buf = ctypes.create_string_buffer(seq.encode())
        L = lib()
        prob = _Problem(ctypes.cast(self._seq_buf, ctypes.c_char_p), dangle, 1 if noGU else 0,
                        ctypes.cast(self._blob_buf, ctypes.c_void_p), None)
        h = ctypes.c_void_p()
        self._raw = load_pfraw(params)
        rc = L.ccj_pf_create(ctypes.byref(prob), self._raw, device, ctypes.byref(h))
        if rc != CCJ_OK:
            raise CCJError(rc, "ccj_pf_create failed (see stderr)")
        self._h = h
        self.energy: Optional[float] = None

    def _check(self, rc: int):
        if rc != CCJ_OK:
            raise CCJError(rc, lib().ccj_pf_last_message(self._h).decode())

    def ccj_pf(self) -> float:
        e = ctypes.c_double()
        self._check(lib().ccj_pf_fill(self._h, ctypes.byref(e)))
        self.energy = e.value
        return e.value

    def W(self) -> list:
        out = (ctypes.c_double * (self.n + 1))()
        self._check(lib().ccj_pf_W(self._h, out))
        return list(out)

    def get2(self, name: str) -> list:
        """One 2-D matrix in canonical order (i = 1..n, j = i..n)."""
        out = (ctypes.c_double * (self.n * (self.n + 1) // 2))()
        self._check(lib().ccj_pf_get2(self._h, PF_MAT2.index(name), out))
        return list(out)

    def get4(self, name: str, i: int, j: int, k: int, l: int) -> int:
        """Matrix4DPF::get: the stored int, 0 outside i <= j < k-1, k <= l."""
        v = ctypes.c_int()
        self._check(lib().ccj_pf_get4(self._h, PF_MAT4.index(name), i, j, k, l, ctypes.byref(v)))
        return v.value

    def hashes(self) -> dict:
        h4 = (ctypes.c_uint64 * len(PF_MAT4))()
        h2 = (ctypes.c_uint64 * len(PF_MAT2))()
        self._check(lib().ccj_pf_hashes(self._h, h4, h2))
        d = {k: "%016x" % v for k, v in zip(PF_MAT4, h4)}
        d.update({k: "%016x" % v for k, v in zip(PF_MAT2, h2)})
        return d

    def exp_hashes(self) -> dict:
        names = lib().ccj_pf_exp_names().decode().split()
        out = (ctypes.c_uint64 * len(names))()
        got = lib().ccj_pf_exp_hashes(self._h, out, len(names))
        if got != len(names):
            raise CCJError(CCJ_E_ARG, "ccj_pf_exp_hashes")
        return {k: "%016x" % v for k, v in zip(names, out)}

    def srand(self, seed: int) -> None:
        """srand(seed) for this context's vrna_urn() generator (rand()/RAND_MAX, like the reference build)."""
        self._check(lib().ccj_pf_srand(self._h, seed))

    def sample(self, count: int) -> list:
        """count x Sample_W(1, n) (stoch_backtrack.cc), continuing this context's rand() stream."""
        buf = ctypes.create_string_buffer(max(count, 1) * (self.n + 1))
        done = ctypes.c_int()
        rc = lib().ccj_pf_sample(self._h, count, buf, ctypes.byref(done))
        got = [buf.raw[s * (self.n + 1): s * (self.n + 1) + self.n].decode() for s in range(done.value)]
        if rc == CCJ_E_PF_SAMPLE:
            raise SampleExit(lib().ccj_pf_last_message(self._h).decode(), got)
        self._check(rc)
        return got

    def fill_ms(self) -> float:
        t = ctypes.c_float()
        self._check(lib().ccj_pf_timing(self._h, ctypes.byref(t)))
        return t.value

    @property
    def PF_KERNELS(self) -> tuple:
        """The four kernel families of kernel_ms / work_model.  Family 2, the P terms, is k_pf_ppush
        (pushed by level, the default) or k_pf_pterm (CCJ_PF_PULL=1); ccj_pf.cc reads the variable on
        every fill, so it is read here at call time too."""
        pull = os.environ.get("CCJ_PF_PULL", "0") not in ("", "0")
        return ("k_pf_iloop", "k_pf_level", "k_pf_pterm" if pull else "k_pf_ppush", "k_pf_diag")

    def set_timing(self, on: bool = True):
        """Event pairs around every launch of the following fills (ccj_pf_set_timing)."""
        self._check(lib().ccj_pf_set_timing(self._h, 1 if on else 0))

    def kernel_ms(self) -> dict:
        """Summed launch durations of the last timed fill per kernel family (ms)."""
        v = (ctypes.c_double * 4)()
        self._check(lib().ccj_pf_kernel_ms(self._h, v))
        return dict(zip(self.PF_KERNELS, v))

    def work_model(self) -> dict:
        """Algorithmic HBM bytes of one fill per kernel family (ccj_pf_work_model)."""
        v = (ctypes.c_double * 4)()
        self._check(lib().ccj_pf_work_model(self._h, v))
        return dict(zip(self.PF_KERNELS, v))

    def close(self):
        if getattr(self, "_h", None):
            lib().ccj_pf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
