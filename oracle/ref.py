"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/jerasure_w8.c header).

ctypes binding for the plain-C Jerasure/gf-complete w=8 restatement in oracle/jerasure_w8.c.
Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; the
product (erasure-codes-prototype_amd/) never imports it.

"Buffers" are 1-D numpy uint8 arrays; a char** is a Python list of such arrays, exactly like the
reference passes char** of B-byte host buffers.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile oracle/jerasure_w8.c -> oracle/build/liboracle.so (gcc, no reference sources)."""
    src = os.path.join(_HERE, "jerasure_w8.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        I = ctypes.c_int
        Lg = ctypes.c_long
        IP = ctypes.POINTER(ctypes.c_int)
        PP = ctypes.POINTER(ctypes.c_void_p)
        L.orc_single_multiply.argtypes = [I, I]
        L.orc_single_divide.argtypes = [I, I]
        L.orc_reed_sol_vandermonde_coding_matrix.argtypes = [I, I]
        L.orc_reed_sol_vandermonde_coding_matrix.restype = IP
        L.orc_cauchy_good_general_coding_matrix.argtypes = [I, I]
        L.orc_cauchy_good_general_coding_matrix.restype = IP
        L.orc_cauchy_original_coding_matrix.argtypes = [I, I]
        L.orc_cauchy_original_coding_matrix.restype = IP
        L.orc_cauchy_n_ones.argtypes = [I]
        L.orc_invert_matrix.argtypes = [IP, IP, I]
        L.orc_matrix_multiply.argtypes = [IP, IP, I, I, I, I]
        L.orc_matrix_multiply.restype = IP
        L.orc_free.argtypes = [P]
        L.orc_region_xor.argtypes = [P, P, Lg]
        L.orc_region_multiply.argtypes = [P, I, Lg, P, I]
        L.orc_matrix_encode.argtypes = [I, I, IP, PP, PP, Lg]
        L.orc_matrix_dotprod.argtypes = [I, IP, IP, I, PP, PP, Lg]
        L.orc_matrix_encode_simd.argtypes = [I, I, IP, PP, PP, Lg]
        L.orc_matrix_decode.argtypes = [I, I, IP, I, IP, PP, PP, Lg]
        L.orc_encode_batch_mt.argtypes = [I, I, IP, P, P, Lg, Lg, I]
        L.orc_decode_batch_mt.argtypes = [I, I, IP, P, P, Lg, Lg, I]
        L.orc_call_seq_batch_mt.argtypes = [P, Lg, P, Lg, Lg, Lg, P, IP, IP, I, I]
        _lib = L
    return _lib


def _ints(vals):
    vals = [int(v) for v in vals]
    return (ctypes.c_int * max(1, len(vals)))(*vals)


def _take(ptr, n):
    if not ptr:
        return None
    out = [ptr[i] for i in range(n)]
    lib().orc_free(ctypes.cast(ptr, ctypes.c_void_p))
    return out


def _ptrs(bufs):
    for b in bufs:
        assert b.dtype == np.uint8 and b.flags["C_CONTIGUOUS"]
    return (ctypes.c_void_p * max(1, len(bufs)))(*[b.ctypes.data for b in bufs])


# ------------------------------------------------------------------ Jerasure-level API (rows a1-a7)

def galois_single_multiply(a: int, b: int) -> int:
    return lib().orc_single_multiply(a, b)


def galois_single_divide(a: int, b: int) -> int:
    return lib().orc_single_divide(a, b)


def reed_sol_vandermonde_coding_matrix(k: int, m: int):
    return _take(lib().orc_reed_sol_vandermonde_coding_matrix(k, m), k * m)


def cauchy_good_general_coding_matrix(k: int, m: int):
    """None for m == 2 (Jerasure cbest_8 table: not recoverable offline -> unpinned)."""
    return _take(lib().orc_cauchy_good_general_coding_matrix(k, m), k * m)


def cauchy_original_coding_matrix(k: int, m: int):
    return _take(lib().orc_cauchy_original_coding_matrix(k, m), k * m)


def cauchy_n_ones(e: int) -> int:
    return lib().orc_cauchy_n_ones(e)


def jerasure_invert_matrix(mat, rows: int):
    """Returns (rc, inverse).  Like the library, the inverse is whatever state Gauss-Jordan
    reached when rc == -1 (the reference ignores rc at erasure_code.cpp:128)."""
    a = _ints(mat)
    inv = (ctypes.c_int * (rows * rows))()
    rc = lib().orc_invert_matrix(a, inv, rows)
    return rc, list(inv)


def jerasure_matrix_multiply(m1, m2, r1, c1, r2, c2):
    return _take(lib().orc_matrix_multiply(_ints(m1), _ints(m2), r1, c1, r2, c2), r1 * c2)


def galois_region_xor(src: np.ndarray, dst: np.ndarray, n: int) -> None:
    lib().orc_region_xor(src.ctypes.data, dst.ctypes.data, n)


def jerasure_matrix_encode(k, m, matrix, data, coding, size):
    lib().orc_matrix_encode(k, m, _ints(matrix), _ptrs(data), _ptrs(coding), size)


def jerasure_matrix_encode_simd(k, m, matrix, data, coding, size):
    lib().orc_matrix_encode_simd(k, m, _ints(matrix), _ptrs(data), _ptrs(coding), size)


def jerasure_matrix_dotprod(k, row, src_ids, dest_id, data, coding, size):
    lib().orc_matrix_dotprod(k, _ints(row), _ints(src_ids) if src_ids else None, dest_id,
                             _ptrs(data) if data else None, _ptrs(coding) if coding else None, size)


def jerasure_matrix_decode(k, m, matrix, row_k_ones, erasures, data, coding, size) -> int:
    return lib().orc_matrix_decode(k, m, _ints(matrix), int(bool(row_k_ones)), _ints(erasures),
                                   _ptrs(data), _ptrs(coding), size)


def encode_batch_mt(k, m, matrix, data: np.ndarray, coding: np.ndarray, B: int, S: int, nthreads: int) -> int:
    """CPU baseline: one jerasure_matrix_encode (SIMD split-table) per stripe over nthreads."""
    return lib().orc_encode_batch_mt(k, m, _ints(matrix), data.ctypes.data, coding.ctypes.data, B, S, nthreads)


def decode_batch_mt(k, m, matrix, stripes: np.ndarray, out: np.ndarray, B: int, S: int, nthreads: int) -> int:
    """CPU baseline: stripe s ([S][k+m][B]) loses block s mod (k+m), rebuilt into out[s] by one
    jerasure_matrix_decode (SIMD region kernels) per stripe over nthreads."""
    return lib().orc_decode_batch_mt(k, m, _ints(matrix), stripes.ctypes.data, out.ctypes.data, B, S, nthreads)


def call_seq_batch_mt(stripes: np.ndarray, out: np.ndarray, patterns, pat_of_stripe, nscr: int, nthreads: int) -> int:
    """CPU baseline of a per-stripe call sequence (bench.py config3 / config4): stripes [S][nb][B], out
    [S][nout][B]; patterns[p] = [(dst, [src ids], [coefs]), ...], each call one jerasure_matrix_encode(kin, 1)
    (SIMD region kernels).  Ids: stripe blocks 0..nb-1, out blocks nb.., then nscr per-thread scratch
    blocks.  Stripe s runs patterns[pat_of_stripe[s]] (pattern 0 when pat_of_stripe is None)."""
    S, nb, B = stripes.shape
    nout = out.shape[1]
    assert out.shape[0] == S and out.shape[2] == B and stripes.flags["C_CONTIGUOUS"] and out.flags["C_CONTIGUOUS"]
    off, packed = [0], []
    for calls in patterns:
        for dst, src, coef in calls:
            assert len(src) == len(coef) and 0 < len(src) <= 256
            assert all(0 <= i < nb + nout + nscr for i in list(src) + [dst])
            packed += [len(src), dst, *src, *coef]
        off.append(len(packed))
    pat = None
    if pat_of_stripe is not None:
        pat = np.ascontiguousarray(pat_of_stripe, dtype=np.int32)
        assert pat.shape == (S,) and pat.min() >= 0 and pat.max() < len(patterns)
    return lib().orc_call_seq_batch_mt(stripes.ctypes.data, nb, out.ctypes.data, nout, B, S,
                                       pat.ctypes.data if pat is not None else None, _ints(off), _ints(packed),
                                       nscr, nthreads)


# ------------------------------------------------------------------ synthetic data

_GOLD = np.uint64(0x9E3779B97F4A7C15)


def splitmix_bytes(seed: int, word_offset: int, nbytes: int) -> np.ndarray:
    """Counter-based bytes: word w (8 bytes, little endian) = splitmix64(seed + (word_offset+w)*golden).
    Bit-identical to the product's device fill (ecg_fill_random)."""
    nw = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        w = np.arange(word_offset, word_offset + nw, dtype=np.uint64)
        z = np.uint64(seed) + w * _GOLD
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()
