"""Python binding of libecg.so (include/ecg.h) — the MI355X erasure-coding engine.

Mirrors the reference's call surface so tests and benches read like the reference's own:
  * Jerasure-level functions (reed_sol_vandermonde_coding_matrix, jerasure_matrix_encode, ...) with
    host buffers (numpy uint8 arrays), as rs.cpp / lrc.cpp / erasure_code.cpp call them;
  * the ErasureCode facade (ec_factory + RSCode / Azu_LRC / ProductCode ... methods) accepting
    either host numpy buffers (reference semantics, synchronous) or HBM-resident torch uint8 CUDA
    tensors (asynchronous on torch's current stream);
  * batched device entry points used by bench.py.

There is no CPU fallback anywhere: if libecg.so is missing or has no GPU to run on, calls raise.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from enum import IntEnum

import numpy as np

try:  # load torch first so libecg binds to the HIP runtime torch already mapped (one runtime per process)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for host-tier use
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ECG_LIB") or os.path.join(_HERE, "lib", "libecg.so")  # ECG_LIB: tuning builds only

ECG_OK = 0
ECG_EUNDECODABLE = -1
ECG_EINVAL = -2
ECG_EHIP = -3
ECG_EUNPINNED = -4
ECG_OPT_NT = 0
ECG_OPT_COLS_PER_WG = 1
ECG_OPT_GRID_MAP = 2
ECG_OPT_ZEROCOPY_BYTES = 3
ECG_OPT_PROGRAM_CACHE = 4
ECG_OPT_MAP_GROUP = 5
ECG_OPT_LAT_DWORD_BYTES = 6
ECG_OPT_CALL_WORKER = 7
ECG_OPT_ROW_SPLIT = 8
ECG_OPT_GRAVEYARD = 9
ECG_OPT_MT1_LDS_PAD = 10
ECG_OPT_COUNT = 11
ECG_MEM_HOST = 0
ECG_MEM_DEVICE = 1


class PlacementRule(IntEnum):  # include/ec/erasure_code.h:31-36 (+ Azure sub-optimal)
    FLAT = 0
    RANDOM = 1
    OPTIMAL = 2
    SUB_OPTIMAL = 3


@dataclass
class RepairPlan:  # include/ec/erasure_code.h:53-58
    local_or_column: bool
    failure_idxs: list
    help_blocks: list

# Every symbol include/ecg.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "ecg_last_error", "ecg_version", "ecg_device_count", "ecg_set_device", "ecg_free", "ecg_program_cache_size", "ecg_program_sets_retiring", "ecg_program_sets_reclaim", "ecg_host_contexts",
    "ecg_host_pinned_xfer_threshold", "ecg_call_worker_stats",
    "ecg_set_option", "ecg_get_option",
    "ecg_reed_sol_vandermonde_coding_matrix", "ecg_cauchy_good_general_coding_matrix",
    "ecg_cauchy_original_coding_matrix", "ecg_cauchy_improve_coding_matrix", "ecg_cauchy_n_ones",
    "ecg_jerasure_invert_matrix", "ecg_jerasure_matrix_multiply", "ecg_galois_region_xor",
    "ecg_jerasure_matrix_encode", "ecg_jerasure_matrix_decode", "ecg_jerasure_matrix_dotprod",
    "ecg_batch_begin", "ecg_batch_flush", "ecg_batch_end", "ecg_batch_defer_host", "ecg_batch_scratch",
    "ecg_batch_last_stats", "ecg_traffic_counters",
    "ecg_dev_matrix_encode", "ecg_dev_matrix_decode", "ecg_matrix_apply_batch", "ecg_matrix_apply_batch_multi",
    "ecg_encode_batch",
    "ecg_decode_batch", "ecg_perform_addition_batch", "ecg_make_decode_matrix", "ecg_region_xor_batch", "ecg_encode_batch_host", "ecg_decode_batch_host",
    "ecg_fill_random",
    "ecg_ec_factory", "ecg_ec_destroy", "ecg_ec_init_coding_parameters", "ecg_ec_get_coding_parameters",
    "ecg_ec_set_memory", "ecg_ec_set_isvertical", "ecg_ec_k", "ecg_ec_m", "ecg_ec_make_encoding_matrix",
    "ecg_ec_check_if_decodable", "ecg_ec_encode", "ecg_ec_decode",
    "ecg_ec_encode_partial_blocks_for_encoding", "ecg_ec_encode_partial_blocks_for_decoding",
    "ecg_ec_perform_addition", "ecg_ec_encode_partial_blocks_for_decoding_with_addition",
    "ecg_ec_encode_partial_blocks_for_encoding_with_addition",
    "ecg_ec_partial_decoding_matrix", "ecg_ec_partial_encoding_matrix",
    "ecg_ec_set_placement_rule", "ecg_ec_set_random_seed", "ecg_ec_generate_partition", "ecg_ec_get_partition",
    "ecg_ec_set_partition", "ecg_ec_grouping_information", "ecg_ec_generate_repair_plan", "ecg_ec_self_information",
    "ecg_ec_bid2gid", "ecg_ec_idxingroup", "ecg_ec_get_group_size", "ecg_ec_bid2rowcol", "ecg_ec_rowcol2bid",
]


class EcgError(RuntimeError):
    def __init__(self, code, what=""):
        msg = f"{what}: ecg status {code}"
        if code == ECG_EHIP:
            msg += f" ({_L.ecg_last_error().decode()})" if _L is not None else ""
        super().__init__(msg)
        self.code = code


class ECTYPE(IntEnum):  # project/include/ec/erasure_code.h:17-29
    RS = 0
    ERS = 1
    AZURE_LRC = 2
    AZURE_LRC_1 = 3
    OPTIMAL_LRC = 4
    OPTIMAL_CAUCHY_LRC = 5
    UNIFORM_CAUCHY_LRC = 6
    PC = 7
    Hierachical_PC = 8
    HV_PC = 9


class _CP(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("k", "m", "l", "g", "k1", "m1", "k2", "m2", "x", "seri_num",
                                          "local_or_column")]


@dataclass
class CodingParameters:  # project/include/ec/erasure_code.h:38-51
    k: int = 0
    m: int = 0
    l: int = 0
    g: int = 0
    k1: int = 0
    m1: int = 0
    k2: int = 0
    m2: int = 0
    x: int = 0
    seri_num: int = 0
    local_or_column: bool = False

    def to_c(self):
        return _CP(self.k, self.m, self.l, self.g, self.k1, self.m1, self.k2, self.m2, self.x, self.seri_num,
                   int(bool(self.local_or_column)))


_L = None


def lib():
    """Load libecg.so (raises if it was not built: the product has no fallback path)."""
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built (run `make -C erasure-codes-prototype_amd`)")
    L = ctypes.CDLL(LIB_PATH)
    I, LL, P, ULL = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_ulonglong
    IP = ctypes.POINTER(ctypes.c_int)
    PP = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "ecg_last_error": ([], ctypes.c_char_p),
        "ecg_version": ([], I),
        "ecg_make_decode_matrix": ([I, I, IP, I, IP, IP, I, IP, IP, I, IP, IP], I),
        "ecg_region_xor_batch": ([P, LL, P, LL, LL, I, P], I),
        "ecg_program_cache_size": ([], I),
        "ecg_program_sets_retiring": ([], I),
        "ecg_program_sets_reclaim": ([], I),
        "ecg_host_contexts": ([], I),
        "ecg_host_pinned_xfer_threshold": ([], LL),
        "ecg_call_worker_stats": ([ctypes.POINTER(LL)] * 3 + [ctypes.POINTER(I)], I),
        "ecg_batch_begin": ([], I),
        "ecg_batch_flush": ([], I),
        "ecg_batch_defer_host": ([I], I),
        "ecg_batch_end": ([], I),
        "ecg_batch_scratch": ([P, ctypes.c_size_t], I),
        "ecg_batch_last_stats": ([ctypes.POINTER(LL)] * 4, I),
        "ecg_traffic_counters": ([ctypes.POINTER(LL)] * 2, I),
        "ecg_device_count": ([], I),
        "ecg_set_device": ([I], I),
        "ecg_free": ([P], None),
        "ecg_set_option": ([I, LL], I),
        "ecg_get_option": ([I], LL),
        "ecg_reed_sol_vandermonde_coding_matrix": ([I, I, I], IP),
        "ecg_cauchy_good_general_coding_matrix": ([I, I, I], IP),
        "ecg_cauchy_original_coding_matrix": ([I, I, I], IP),
        "ecg_cauchy_improve_coding_matrix": ([I, I, I, IP], None),
        "ecg_cauchy_n_ones": ([I, I], I),
        "ecg_jerasure_invert_matrix": ([IP, IP, I, I], I),
        "ecg_jerasure_matrix_multiply": ([IP, IP, I, I, I, I, I], IP),
        "ecg_galois_region_xor": ([P, P, I], I),
        "ecg_jerasure_matrix_encode": ([I, I, I, IP, PP, PP, I], I),
        "ecg_jerasure_matrix_decode": ([I, I, I, IP, I, IP, PP, PP, I], I),
        "ecg_jerasure_matrix_dotprod": ([I, I, IP, IP, I, PP, PP, I], I),
        "ecg_dev_matrix_encode": ([I, I, IP, PP, PP, LL, P], I),
        "ecg_dev_matrix_decode": ([I, I, IP, I, IP, PP, PP, LL, P], I),
        "ecg_matrix_apply_batch": ([I, I, IP, IP, IP, P, LL, LL, P, LL, LL, LL, I, P], I),
        "ecg_matrix_apply_batch_multi": ([I, I, I, IP, IP, IP, P, P, P, LL, LL, P, LL, LL, LL, I, P], I),
        "ecg_encode_batch": ([I, I, IP, P, LL, LL, P, LL, LL, LL, I, P], I),
        "ecg_decode_batch": ([I, I, IP, I, IP, I, P, P, LL, LL, P, LL, LL, LL, I, P], I),
        "ecg_perform_addition_batch": ([I, I, P, LL, LL, P, LL, LL, LL, I, P], I),
        "ecg_encode_batch_host": ([I, I, IP, P, LL, LL, P, LL, LL, LL, I, I], I),
        "ecg_decode_batch_host": ([I, I, IP, I, IP, P, LL, LL, P, LL, LL, LL, I, I], I),
        "ecg_fill_random": ([P, LL, ULL, ULL, P], I),
        "ecg_ec_factory": ([I, ctypes.POINTER(_CP)], P),
        "ecg_ec_destroy": ([P], None),
        "ecg_ec_init_coding_parameters": ([P, ctypes.POINTER(_CP)], I),
        "ecg_ec_get_coding_parameters": ([P, ctypes.POINTER(_CP)], I),
        "ecg_ec_set_memory": ([P, I, P], I),
        "ecg_ec_set_isvertical": ([P, I], I),
        "ecg_ec_k": ([P], I),
        "ecg_ec_m": ([P], I),
        "ecg_ec_make_encoding_matrix": ([P, IP], I),
        "ecg_ec_check_if_decodable": ([P, IP, I], I),
        "ecg_ec_encode": ([P, PP, PP, I], I),
        "ecg_ec_decode": ([P, PP, PP, I, IP, I], I),
        "ecg_ec_encode_partial_blocks_for_encoding": ([P, PP, PP, I, IP, I, IP, I], I),
        "ecg_ec_encode_partial_blocks_for_decoding": ([P, PP, PP, I, IP, I, IP, I, IP, I], I),
        "ecg_ec_perform_addition": ([P, PP, PP, I, I, I], I),
        "ecg_ec_encode_partial_blocks_for_decoding_with_addition": ([P, PP, PP, I, PP, I, IP, I, IP, I, IP, I], I),
        "ecg_ec_encode_partial_blocks_for_encoding_with_addition": ([P, PP, PP, I, PP, I, IP, I, IP, I], I),
        "ecg_ec_partial_decoding_matrix": ([P, IP, I, IP, I, IP, I, IP, I], I),
        "ecg_ec_partial_encoding_matrix": ([P, IP, I, IP, I, IP, I], I),
        "ecg_ec_set_placement_rule": ([P, I], I),
        "ecg_ec_set_random_seed": ([P, ULL], I),
        "ecg_ec_generate_partition": ([P], I),
        "ecg_ec_get_partition": ([P, IP, I], I),
        "ecg_ec_set_partition": ([P, IP, I], I),
        "ecg_ec_grouping_information": ([P, IP, I], I),
        "ecg_ec_generate_repair_plan": ([P, IP, I, IP, I, IP], I),
        "ecg_ec_self_information": ([P, ctypes.c_char_p, I], I),
        "ecg_ec_bid2gid": ([P, I], I),
        "ecg_ec_idxingroup": ([P, I], I),
        "ecg_ec_get_group_size": ([P, I, IP], I),
        "ecg_ec_bid2rowcol": ([P, I, IP, IP], I),
        "ecg_ec_rowcol2bid": ([P, I, I], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _L = L
    return L


def host_pinned_xfer_threshold():
    """ecg_host_pinned_xfer_threshold: bytes above which the HIP runtime pins a pageable copy itself
    (GPU_PINNED_MIN_XFER_SIZE; default 1 MiB); -1 if the variable is malformed."""
    return lib().ecg_host_pinned_xfer_threshold()


def call_worker_stats():
    """ecg_call_worker_stats of the current device: {calls, launches, relaunches, disabled}."""
    v = [ctypes.c_longlong(0) for _ in range(3)]
    dis = ctypes.c_int(0)
    _check(lib().ecg_call_worker_stats(*[ctypes.byref(x) for x in v], ctypes.byref(dis)), "call_worker_stats")
    return {"calls": v[0].value, "launches": v[1].value, "relaunches": v[2].value, "disabled": bool(dis.value)}


def set_option(option, value):
    """Kernel tuning knob (include/ecg.h ECG_OPT_*); never changes results."""
    return _check(lib().ecg_set_option(option, value), "set_option")


def get_option(option):
    return lib().ecg_get_option(option)


def _ints(vals):
    vals = [int(v) for v in vals]
    return (ctypes.c_int * max(1, len(vals)))(*vals)


def _take(ptr, n):
    if not ptr:
        return None
    out = [ptr[i] for i in range(n)]
    lib().ecg_free(ctypes.cast(ptr, ctypes.c_void_p))
    return out


def _is_dev(b):
    return torch is not None and isinstance(b, torch.Tensor) and b.is_cuda


def _addr(b):
    if b is None:
        return None
    if _is_dev(b):
        assert b.dtype == torch.uint8 and b.is_contiguous()
        return b.data_ptr()
    assert isinstance(b, np.ndarray) and b.dtype == np.uint8 and b.flags["C_CONTIGUOUS"], "uint8 C-contiguous"
    return b.ctypes.data


def _ptrs(bufs):
    return (ctypes.c_void_p * max(1, len(bufs)))(*[_addr(b) for b in bufs])


def _stream(stream):
    if stream is not None:
        return ctypes.c_void_p(stream)
    if torch is not None and torch.cuda.is_available():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    return None


def _check(rc, what):
    if rc < 0:
        raise EcgError(rc, what)
    return rc


# ------------------------------------------------------------------ tier 1 (Jerasure-compatible)

def reed_sol_vandermonde_coding_matrix(k, m, w=8):
    return _take(lib().ecg_reed_sol_vandermonde_coding_matrix(k, m, w), k * m)


def cauchy_good_general_coding_matrix(k, m, w=8):
    return _take(lib().ecg_cauchy_good_general_coding_matrix(k, m, w), k * m)


def cauchy_original_coding_matrix(k, m, w=8):
    return _take(lib().ecg_cauchy_original_coding_matrix(k, m, w), k * m)


def cauchy_n_ones(e, w=8):
    return lib().ecg_cauchy_n_ones(e, w)


def jerasure_invert_matrix(mat, rows, w=8):
    a = _ints(mat)
    inv = (ctypes.c_int * (rows * rows))()
    rc = lib().ecg_jerasure_invert_matrix(a, inv, rows, w)
    return rc, list(inv)


def jerasure_matrix_multiply(m1, m2, r1, c1, r2, c2, w=8):
    return _take(lib().ecg_jerasure_matrix_multiply(_ints(m1), _ints(m2), r1, c1, r2, c2, w), r1 * c2)


def galois_region_xor(src, dst, n):
    return _check(lib().ecg_galois_region_xor(_addr(src), _addr(dst), n), "galois_region_xor")


def jerasure_matrix_encode(k, m, matrix, data, coding, size, w=8):
    return _check(lib().ecg_jerasure_matrix_encode(k, m, w, _ints(matrix), _ptrs(data), _ptrs(coding), size),
                  "jerasure_matrix_encode")


def jerasure_matrix_dotprod(k, matrix_row, src_ids, dest_id, data, coding, size, w=8):
    """jerasure_matrix_dotprod (host buffers): one coefficient row into block dest_id."""
    return _check(lib().ecg_jerasure_matrix_dotprod(k, w, _ints(matrix_row), _ints(src_ids) if src_ids else None,
                                                     dest_id, _ptrs(data) if data else None,
                                                     _ptrs(coding) if coding else None, size), "jerasure_matrix_dotprod")


def jerasure_matrix_decode(k, m, matrix, row_k_ones, erasures, data, coding, size, w=8):
    return lib().ecg_jerasure_matrix_decode(k, m, w, _ints(matrix), int(bool(row_k_ones)), _ints(erasures),
                                            _ptrs(data), _ptrs(coding), size)


# ------------------------------------------------------------------ tier 2 (device / batched)

class batch:
    """Deferred-batch scope (ecg_batch_begin / ecg_batch_end): per-stripe device-tier calls made by this
    thread inside the `with` block are recorded and launched on exit, one launch per plan and op where no
    data dependence orders the calls apart.  `scratch(t)` declares a device tensor (or (ptr, nbytes))
    scratch: partial results written there and read later in the scope are composed away.  host=True also
    defers host-tier calls (ecg_batch_defer_host): their outputs are written when the scope flushes."""

    def __init__(self, host=False):
        self.host = host

    def __enter__(self):
        _check(lib().ecg_batch_begin(), "batch_begin")
        if self.host:
            rc = lib().ecg_batch_defer_host(1)
            if rc:
                lib().ecg_batch_end()
                _check(rc, "batch_defer_host")
        return self

    def flush(self):
        _check(lib().ecg_batch_flush(), "batch_flush")

    def scratch(self, t, nbytes=None):
        batch_scratch(t, nbytes)

    def __exit__(self, exc_type, exc, tb):
        rc = lib().ecg_batch_end()
        if exc_type is None:
            _check(rc, "batch_end")
        return False


def batch_scratch(t, nbytes=None):
    """ecg_batch_scratch: a torch tensor (its whole storage span) or a device address + nbytes."""
    if nbytes is None:
        ptr, nbytes = t.data_ptr(), t.numel() * t.element_size()
    else:
        ptr = t if isinstance(t, int) else t.data_ptr()
    _check(lib().ecg_batch_scratch(ctypes.c_void_p(ptr), nbytes), "batch_scratch")


def batch_last_stats():
    """What this thread's last flush did: {recorded, composed, launches, materialised}."""
    v = [ctypes.c_longlong(0) for _ in range(4)]
    _check(lib().ecg_batch_last_stats(*[ctypes.byref(x) for x in v]), "batch_last_stats")
    return dict(zip(("recorded", "composed", "launches", "materialised"), (x.value for x in v)))


def traffic_counters():
    """Process-wide {launches, bytes}: region-product kernels launched so far and the bytes they move as planned
    (S * B * (row tiles * k + m) per launch).  Differences over a region of calls give its executed traffic."""
    v = [ctypes.c_longlong(0) for _ in range(2)]
    _check(lib().ecg_traffic_counters(*[ctypes.byref(x) for x in v]), "traffic_counters")
    return {"launches": v[0].value, "bytes": v[1].value}


def dev_matrix_encode(k, m, matrix, data, coding, B, stream=None):
    return _check(lib().ecg_dev_matrix_encode(k, m, _ints(matrix), _ptrs(data), _ptrs(coding), B, _stream(stream)),
                  "dev_matrix_encode")


def dev_matrix_decode(k, m, matrix, row_k_ones, erasures, data, coding, B, stream=None):
    return lib().ecg_dev_matrix_decode(k, m, _ints(matrix), int(bool(row_k_ones)), _ints(erasures), _ptrs(data),
                                       _ptrs(coding), B, _stream(stream))


def _strides(t):
    """(stripe stride, block stride) in bytes for a [S][n][B] uint8 tensor view."""
    return t.stride(0), t.stride(1)


def encode_batch(k, m, matrix, d_in, d_out, stream=None):
    """d_in: [S][k][B] uint8 CUDA tensor (any strides, 16-B aligned rows); d_out: [S][m][B]."""
    S, _, B = d_in.shape
    iss, ibs = _strides(d_in)
    oss, obs = _strides(d_out)
    return _check(lib().ecg_encode_batch(k, m, _ints(matrix), d_in.data_ptr(), iss, ibs, d_out.data_ptr(), oss, obs,
                                         B, S, _stream(stream)), "encode_batch")


def decode_batch(k, m, matrix, row_k_ones, patterns, stripes, out=None, pattern_of_stripe=None, stream=None):
    """stripes: [S][k+m][B]; patterns: list of erasure lists; pattern_of_stripe: int32 CUDA tensor [S]."""
    S, _, B = stripes.shape
    flat = []
    for p in patterns:
        flat += list(p) + [-1]
    ss, bs = _strides(stripes)
    oss, obs = _strides(out) if out is not None else (0, 0)
    pos = pattern_of_stripe.data_ptr() if pattern_of_stripe is not None else None
    return _check(lib().ecg_decode_batch(k, m, _ints(matrix), int(bool(row_k_ones)), _ints(flat), len(patterns), pos,
                                         stripes.data_ptr(), ss, bs, out.data_ptr() if out is not None else None,
                                         oss, obs, B, S, _stream(stream)), "decode_batch")


def matrix_apply_batch(coef, src_ids, dst_ids, d_in, d_out, stream=None):
    """coef: n_out x n_in (flat or nested); d_in [S][*][B], d_out [S][*][B]."""
    coef = np.asarray(coef, dtype=np.int64).reshape(len(dst_ids), len(src_ids))
    S, _, B = d_in.shape
    iss, ibs = _strides(d_in)
    oss, obs = _strides(d_out)
    return _check(lib().ecg_matrix_apply_batch(len(src_ids), len(dst_ids), _ints(coef.ravel()), _ints(src_ids),
                                               _ints(dst_ids), d_in.data_ptr(), iss, ibs, d_out.data_ptr(), oss, obs,
                                               B, S, _stream(stream)), "matrix_apply_batch")


class Programs:
    """Same-shape programs (coef [n_out][n_in], src_ids, dst_ids) packed once into the C arrays
    matrix_apply_batch_multi passes; re-packing per call is most of a launch's Python-side cost, which
    matters when a batch is issued in chunks (ecg_dist.pipelined_ring_repair)."""

    def __init__(self, programs):
        programs = list(programs)
        if not programs:
            raise EcgError(ECG_EINVAL, "matrix_apply_batch_multi: no programs")
        self.n_prog = len(programs)
        self.k_in, self.m_out = len(programs[0][1]), len(programs[0][2])
        coefs, srcs, dsts = [], [], []
        for coef, src, dst in programs:
            if len(src) != self.k_in or len(dst) != self.m_out:
                raise EcgError(ECG_EINVAL, "matrix_apply_batch_multi: programs differ in shape")
            c = np.asarray(coef, dtype=np.int64).reshape(self.m_out, self.k_in)
            coefs += list(c.ravel())
            srcs += list(src)
            dsts += list(dst)
        self.coefs, self.srcs, self.dsts = _ints(coefs), _ints(srcs), _ints(dsts)


def matrix_apply_batch_multi(programs, d_in, d_out, prog_of_stripe=None, stripe_of=None, n_launch=None,
                             stream=None):
    """programs: list of (coef [n_out][n_in], src_ids, dst_ids), all of the same shape, or a Programs.
    Launch stripe i runs programs[prog_of_stripe[i]] on stripe stripe_of[i] (int32 CUDA tensors; None =
    identity)."""
    P = programs if isinstance(programs, Programs) else Programs(programs)
    _, _, B = d_in.shape
    S = n_launch if n_launch is not None else (stripe_of.numel() if stripe_of is not None else d_in.shape[0])
    iss, ibs = _strides(d_in)
    oss, obs = _strides(d_out)
    return _check(lib().ecg_matrix_apply_batch_multi(
        P.n_prog, P.k_in, P.m_out, P.coefs, P.srcs, P.dsts,
        prog_of_stripe.data_ptr() if prog_of_stripe is not None else None,
        stripe_of.data_ptr() if stripe_of is not None else None,
        d_in.data_ptr(), iss, ibs, d_out.data_ptr(), oss, obs, B, S, _stream(stream)), "matrix_apply_batch_multi")


def make_decode_matrix(k, m, matrix, row_k_ones, erasures):
    """jerasure_matrix_decode composed into one map: (src_ids, dst_ids, coef[n_dst][n_src]) or raises."""
    n_src, n_dst = ctypes.c_int(0), ctypes.c_int(0)
    er = _ints(list(erasures) + ([-1] if not erasures or erasures[-1] != -1 else []))
    _check(lib().ecg_make_decode_matrix(k, m, _ints(matrix), int(bool(row_k_ones)), er, None, 0, ctypes.byref(n_src),
                                        None, 0, ctypes.byref(n_dst), None), "make_decode_matrix")
    ns, nd = n_src.value, n_dst.value
    src, dst, coef = (ctypes.c_int * max(1, ns))(), (ctypes.c_int * max(1, nd))(), (ctypes.c_int * max(1, ns * nd))()
    _check(lib().ecg_make_decode_matrix(k, m, _ints(matrix), int(bool(row_k_ones)), er, src, ns, ctypes.byref(n_src),
                                        dst, nd, ctypes.byref(n_dst), coef), "make_decode_matrix")
    return list(src)[:ns], list(dst)[:nd], [list(coef)[i * ns:(i + 1) * ns] for i in range(nd)]


def region_xor_batch(d_src, d_dst, stream=None):
    """dst[s] ^= src[s] for every row s of two [S][nbytes] uint8 CUDA tensors (galois_region_xor, batched)."""
    S, n = d_src.shape
    return _check(lib().ecg_region_xor_batch(d_src.data_ptr(), d_src.stride(0), d_dst.data_ptr(), d_dst.stride(0), n, S,
                                             _stream(stream)), "region_xor_batch")


def perform_addition_batch(block_num, parity_num, d_in, d_out, stream=None):
    S, _, B = d_in.shape
    iss, ibs = _strides(d_in)
    oss, obs = _strides(d_out)
    return _check(lib().ecg_perform_addition_batch(block_num, parity_num, d_in.data_ptr(), iss, ibs, d_out.data_ptr(),
                                                   oss, obs, B, S, _stream(stream)), "perform_addition_batch")


def _host_strides(a):
    """(stripe stride, block stride) in bytes of a [S][n][B] host array (numpy or pinned torch CPU)."""
    if isinstance(a, np.ndarray):
        return a.strides[0], a.strides[1], a.ctypes.data
    return a.stride(0), a.stride(1), a.data_ptr()


def encode_batch_host(k, m, matrix, h_in, h_out, chunk_stripes=0):
    """Host-resident RS/any-matrix encode through the H2D -> kernel -> D2H pipeline.  h_in [S][k][B],
    h_out [S][m][B] (numpy or pinned torch CPU uint8)."""
    S, _, B = h_in.shape
    iss, ibs, ip = _host_strides(h_in)
    oss, obs, op = _host_strides(h_out)
    return _check(lib().ecg_encode_batch_host(k, m, _ints(matrix), ip, iss, ibs, op, oss, obs, B, S, chunk_stripes),
                  "encode_batch_host")


def decode_batch_host(k, m, matrix, row_k_ones, erasures, h_stripes, h_out=None, chunk_stripes=0):
    S, _, B = h_stripes.shape
    ss, bs, sp = _host_strides(h_stripes)
    oss, obs, op = _host_strides(h_out) if h_out is not None else (0, 0, None)
    return _check(lib().ecg_decode_batch_host(k, m, _ints(matrix), int(bool(row_k_ones)), _ints(list(erasures) + [-1]),
                                              sp, ss, bs, op, oss, obs, B, S, chunk_stripes), "decode_batch_host")


def fill_random(t, seed, word_offset=0, stream=None):
    """Fill a CUDA uint8 tensor with the splitmix64 counter stream (same bytes as oracle.ref.splitmix_bytes)."""
    return _check(lib().ecg_fill_random(t.data_ptr(), t.numel(), seed, word_offset, _stream(stream)), "fill_random")


# ------------------------------------------------------------------ tier 3 (ErasureCode facade)

class ErasureCode:
    """Handle on one C++ ErasureCode object (project/include/ec/erasure_code.h:60-129)."""

    def __init__(self, handle):
        if not handle:
            raise EcgError(ECG_EINVAL, "ec_factory")
        self._h = ctypes.c_void_p(handle)
        self._mem = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _L is not None:
            _L.ecg_ec_destroy(h)
            self._h = None

    # --- parameters
    @property
    def k(self):
        return lib().ecg_ec_k(self._h)

    @property
    def m(self):
        return lib().ecg_ec_m(self._h)

    def init_coding_parameters(self, cp: CodingParameters):
        c = cp.to_c()
        _check(lib().ecg_ec_init_coding_parameters(self._h, ctypes.byref(c)), "init_coding_parameters")

    def get_coding_parameters(self) -> CodingParameters:
        c = _CP()
        _check(lib().ecg_ec_get_coding_parameters(self._h, ctypes.byref(c)), "get_coding_parameters")
        return CodingParameters(c.k, c.m, c.l, c.g, c.k1, c.m1, c.k2, c.m2, c.x, c.seri_num, bool(c.local_or_column))

    def set_isvertical(self, v: bool):
        _check(lib().ecg_ec_set_isvertical(self._h, int(bool(v))), "set_isvertical")

    def make_encoding_matrix(self, rows=None):
        rows = self.m if rows is None else rows
        out = (ctypes.c_int * max(1, rows * self.k))()
        _check(lib().ecg_ec_make_encoding_matrix(self._h, out), "make_encoding_matrix")
        return list(out)

    def check_if_decodable(self, failure_idxs):
        return _check(lib().ecg_ec_check_if_decodable(self._h, _ints(failure_idxs), len(failure_idxs)),
                      "check_if_decodable") == 1

    # --- memory tier follows the buffers: numpy -> host (synchronous), torch CUDA -> device (async)
    def _bind(self, bufs, stream=None):
        dev = any(_is_dev(b) for b in bufs if b is not None)
        mem = ECG_MEM_DEVICE if dev else ECG_MEM_HOST
        st = _stream(stream) if dev else None
        _check(lib().ecg_ec_set_memory(self._h, mem, st), "set_memory")

    def encode(self, data_ptrs, coding_ptrs, block_size, stream=None):
        self._bind(list(data_ptrs) + list(coding_ptrs), stream)
        return _check(lib().ecg_ec_encode(self._h, _ptrs(data_ptrs), _ptrs(coding_ptrs), block_size), "encode")

    def decode(self, data_ptrs, coding_ptrs, block_size, erasures, failed_num, stream=None):
        """erasures: list (-1 terminated like the reference; the LRC local path reads group_id at
        erasures[failed_num] and overwrites it with -1, lrc.cpp:35-38 — mirrored into the list)."""
        self._bind(list(data_ptrs) + list(coding_ptrs), stream)
        er = _ints(erasures)
        rc = lib().ecg_ec_decode(self._h, _ptrs(data_ptrs), _ptrs(coding_ptrs), block_size, er, failed_num)
        for i in range(len(erasures)):
            erasures[i] = er[i]
        return rc

    def encode_partial_blocks_for_encoding(self, data_ptrs, coding_ptrs, block_size, data_idxs, parity_idxs,
                                           stream=None):
        self._bind(list(data_ptrs) + list(coding_ptrs), stream)
        return _check(lib().ecg_ec_encode_partial_blocks_for_encoding(
            self._h, _ptrs(data_ptrs), _ptrs(coding_ptrs), block_size, _ints(data_idxs), len(data_idxs),
            _ints(parity_idxs), len(parity_idxs)), "encode_partial_blocks_for_encoding")

    def encode_partial_blocks_for_decoding(self, data_ptrs, coding_ptrs, block_size, local_survivor_idxs,
                                           survivor_idxs, failure_idxs, stream=None):
        self._bind(list(data_ptrs) + list(coding_ptrs), stream)
        return _check(lib().ecg_ec_encode_partial_blocks_for_decoding(
            self._h, _ptrs(data_ptrs), _ptrs(coding_ptrs), block_size, _ints(local_survivor_idxs),
            len(local_survivor_idxs), _ints(survivor_idxs), len(survivor_idxs), _ints(failure_idxs),
            len(failure_idxs)), "encode_partial_blocks_for_decoding")

    def perform_addition(self, data_ptrs, coding_ptrs, block_size, block_num, parity_num, stream=None):
        self._bind(list(data_ptrs) + list(coding_ptrs), stream)
        return lib().ecg_ec_perform_addition(self._h, _ptrs(data_ptrs), _ptrs(coding_ptrs), block_size, block_num,
                                             parity_num)

    def encode_partial_blocks_for_decoding_with_addition(self, local_ptrs, partial_ptrs, out_ptrs, block_size,
                                                         local_survivor_idxs, survivor_idxs, failure_idxs,
                                                         stream=None):
        """The main proxy's own partial + perform_addition of the helpers' partials in one pass
        (handle_repair.cpp:371-376)."""
        self._bind(list(local_ptrs) + list(partial_ptrs) + list(out_ptrs), stream)
        return _check(lib().ecg_ec_encode_partial_blocks_for_decoding_with_addition(
            self._h, _ptrs(local_ptrs), _ptrs(partial_ptrs), len(partial_ptrs), _ptrs(out_ptrs), block_size,
            _ints(local_survivor_idxs), len(local_survivor_idxs), _ints(survivor_idxs), len(survivor_idxs),
            _ints(failure_idxs), len(failure_idxs)), "encode_partial_blocks_for_decoding_with_addition")

    def encode_partial_blocks_for_encoding_with_addition(self, local_ptrs, partial_ptrs, out_ptrs, block_size,
                                                         data_idxs, parity_idxs, stream=None):
        """The parity proxy's own partial encoding + perform_addition of the helpers' partials in one
        pass (handle_merge.cpp:159,319)."""
        self._bind(list(local_ptrs) + list(partial_ptrs) + list(out_ptrs), stream)
        return _check(lib().ecg_ec_encode_partial_blocks_for_encoding_with_addition(
            self._h, _ptrs(local_ptrs), _ptrs(partial_ptrs), len(partial_ptrs), _ptrs(out_ptrs), block_size,
            _ints(data_idxs), len(data_idxs), _ints(parity_idxs), len(parity_idxs)),
            "encode_partial_blocks_for_encoding_with_addition")

    # --- planning hooks (batched repair / merge)
    def partial_decoding_matrix(self, local_survivor_idxs, survivor_idxs, failure_idxs):
        cap = max(1, len(failure_idxs) * len(local_survivor_idxs))
        out = (ctypes.c_int * cap)()
        _check(lib().ecg_ec_partial_decoding_matrix(self._h, _ints(local_survivor_idxs), len(local_survivor_idxs),
                                                    _ints(survivor_idxs), len(survivor_idxs), _ints(failure_idxs),
                                                    len(failure_idxs), out, cap), "partial_decoding_matrix")
        return list(out)[:len(failure_idxs) * len(local_survivor_idxs)]

    def partial_encoding_matrix(self, data_idxs, parity_idxs):
        cap = max(1, len(data_idxs) * len(parity_idxs))
        out = (ctypes.c_int * cap)()
        _check(lib().ecg_ec_partial_encoding_matrix(self._h, _ints(data_idxs), len(data_idxs), _ints(parity_idxs),
                                                    len(parity_idxs), out, cap), "partial_encoding_matrix")
        return list(out)[:len(data_idxs) * len(parity_idxs)]


    # --- partitioning and repair planning (csrc/planning.cpp)
    @property
    def placement_rule(self):
        return self._rule if hasattr(self, "_rule") else PlacementRule.OPTIMAL

    @placement_rule.setter
    def placement_rule(self, rule):
        _check(lib().ecg_ec_set_placement_rule(self._h, int(rule)), "placement_rule")
        self._rule = PlacementRule(int(rule))

    def set_random_seed(self, seed):
        _check(lib().ecg_ec_set_random_seed(self._h, seed & ((1 << 64) - 1)), "set_random_seed")

    def generate_partition(self):  # erasure_code.cpp:159-169
        _check(lib().ecg_ec_generate_partition(self._h), "generate_partition")
        return self.partition_plan

    @staticmethod
    def _call_sized(fn, what):
        n = _check(fn(None, 0), what)
        buf = (ctypes.c_int * max(1, n))()
        _check(fn(buf, n), what)
        return list(buf)[:n]

    @staticmethod
    def _lists(v, at):
        n = v[at]
        at += 1
        out = []
        for _ in range(n):
            sz = v[at]
            out.append(v[at + 1:at + 1 + sz])
            at += 1 + sz
        return out, at

    @property
    def partition_plan(self):
        v = self._call_sized(lambda b, c: lib().ecg_ec_get_partition(self._h, b, c), "get_partition")
        return self._lists(v, 0)[0]

    @partition_plan.setter
    def partition_plan(self, plan):
        flat = [len(plan)]
        for part in plan:
            flat += [len(part)] + list(part)
        _check(lib().ecg_ec_set_partition(self._h, _ints(flat), len(flat)), "set_partition")

    def grouping_information(self):  # LRC only (lrc.h:73)
        v = self._call_sized(lambda b, c: lib().ecg_ec_grouping_information(self._h, b, c), "grouping_information")
        return self._lists(v, 0)[0]

    def generate_repair_plan(self, failure_idxs):
        """Returns (decodable, [RepairPlan]) like the reference's bool + out-parameter."""
        dec = ctypes.c_int(0)
        fi = _ints(failure_idxs)
        v = self._call_sized(lambda b, c: lib().ecg_ec_generate_repair_plan(self._h, fi, len(failure_idxs), b, c,
                                                                            ctypes.byref(dec)),
                             "generate_repair_plan")
        plans, at = [], 1
        for _ in range(v[0]):
            loc, nf = bool(v[at]), v[at + 1]
            fails = v[at + 2:at + 2 + nf]
            helps, at = self._lists(v, at + 2 + nf)
            plans.append(RepairPlan(loc, fails, helps))
        return bool(dec.value), plans

    def self_information(self):
        n = _check(lib().ecg_ec_self_information(self._h, None, 0), "self_information")
        buf = ctypes.create_string_buffer(n + 1)
        lib().ecg_ec_self_information(self._h, buf, n + 1)
        return buf.value.decode()


def ec_factory(ec_type, cp: CodingParameters) -> ErasureCode:  # project/src/metadata.cpp:48-77
    c = cp.to_c()
    return ErasureCode(lib().ecg_ec_factory(int(ec_type), ctypes.byref(c)))
