"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/jerasure_w8.c header; "parity unpinned" against real
Jerasure).  Pure-Python restatement of the reference's EC class behaviour on top of oracle/ref.py:
matrix construction, block-index remaps, partial coding and decode control flow.  Every method cites
the reference line it follows (paths relative to /root/reference/project).

Buffers are numpy uint8 arrays; char** is a list of them.  Matrices are flat Python int lists, the
reference's `int*` convention.  Used only by tests/ as the checker.
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import IntEnum

import numpy as np

from . import ref as J


class ECTYPE(IntEnum):  # include/ec/erasure_code.h:17-29
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


@dataclass
class CodingParameters:  # include/ec/erasure_code.h:38-51
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


class UnpinnedError(RuntimeError):
    """Raised where the reference depends on a Jerasure table not recoverable offline (cbest_8)."""


def _cauchy(k, m):
    M = J.cauchy_good_general_coding_matrix(k, m)
    if M is None:
        raise UnpinnedError(f"cauchy_good_general_coding_matrix({k},{m}) uses Jerasure's cbest_8 table")
    return M


# ==================================================================== ErasureCode base
class ErasureCode:
    w = 8

    def __init__(self, k=6, m=3):  # erasure_code.h:71-79
        self.k = k
        self.m = m
        self.local_or_column = False

    def init_coding_parameters(self, cp):  # erasure_code.cpp:5-10
        self.k = cp.k
        self.m = cp.m
        self.local_or_column = cp.local_or_column

    # erasure_code.cpp:30-35
    @staticmethod
    def get_full_matrix(matrix, kk):
        for i in range(kk):
            matrix[i * kk + i] = 1

    # erasure_code.cpp:37-47
    @staticmethod
    def make_submatrix_by_rows(cols, matrix, new_matrix, block_idxs):
        for i, j in enumerate(block_idxs):
            new_matrix[i * cols:(i + 1) * cols] = matrix[j * cols:(j + 1) * cols]

    # erasure_code.cpp:49-61
    @staticmethod
    def make_submatrix_by_cols(cols, rows, matrix, new_matrix, block_idxs):
        n = len(block_idxs)
        for i, j in enumerate(block_idxs):
            for u in range(rows):
                new_matrix[u * n + i] = matrix[u * cols + j]

    # erasure_code.cpp:70-94
    def perform_addition(self, data_ptrs, coding_ptrs, block_size, block_num, parity_num):
        if block_num % parity_num != 0:
            return
        per = block_num // parity_num
        data = []
        for i in range(parity_num):
            for j in range(per):
                data.append(data_ptrs[j * parity_num + i])
        for i in range(parity_num):
            J.jerasure_matrix_encode(per, 1, [1] * per, data[i * per:(i + 1) * per], [coding_ptrs[i]], block_size)

    # erasure_code.cpp:97-111
    def encode_partial_blocks_for_encoding_(self, k_, full_matrix, data_ptrs, coding_ptrs, block_size,
                                            data_idxs, parity_idxs):
        nb = len(data_idxs)
        npar = len(parity_idxs)
        matrix = [0] * (npar * k_)
        self.make_submatrix_by_rows(k_, full_matrix, matrix, parity_idxs)
        new_matrix = [1] * (npar * nb)
        self.make_submatrix_by_cols(k_, npar, matrix, new_matrix, data_idxs)
        J.jerasure_matrix_encode(nb, npar, new_matrix, data_ptrs, coding_ptrs, block_size)

    # erasure_code.cpp:113-150
    def encode_partial_blocks_for_decoding_(self, k_, full_matrix, data_ptrs, coding_ptrs, block_size,
                                            local_survivor_idxs, survivor_idxs, failure_idxs):
        nl = len(local_survivor_idxs)
        nf = len(failure_idxs)
        fm = [0] * (nf * k_)
        sm = [0] * (k_ * k_)
        self.make_submatrix_by_rows(k_, full_matrix, fm, failure_idxs)
        self.make_submatrix_by_rows(k_, full_matrix, sm, survivor_idxs)
        _rc, inv = J.jerasure_invert_matrix(sm, k_)  # return value ignored, erasure_code.cpp:128
        dec = J.jerasure_matrix_multiply(fm, inv, nf, k_, k_, k_)
        enc = [0] * (nf * nl)
        for i, a in enumerate(local_survivor_idxs):
            idx = 0
            for b in survivor_idxs:
                if a == b:
                    break
                idx += 1
            for u in range(nf):
                enc[u * nl + i] = dec[u * k_ + idx]
        J.jerasure_matrix_encode(nl, nf, enc, data_ptrs, coding_ptrs, block_size)


# ==================================================================== RS / ERS (rs.cpp)
class RSCode(ErasureCode):
    def make_encoding_matrix(self):  # rs.cpp:5-18
        return J.reed_sol_vandermonde_coding_matrix(self.k, self.m)

    def encode(self, data_ptrs, coding_ptrs, block_size):  # rs.cpp:20-25
        J.jerasure_matrix_encode(self.k, self.m, self.make_encoding_matrix(), data_ptrs, coding_ptrs, block_size)

    def decode(self, data_ptrs, coding_ptrs, block_size, erasures, failed_num):  # rs.cpp:27-42
        if failed_num > self.m:
            return -1
        M = J.reed_sol_vandermonde_coding_matrix(self.k, self.m)  # NB: plain RS even for ERS
        return J.jerasure_matrix_decode(self.k, self.m, M, failed_num, erasures, data_ptrs, coding_ptrs,
                                        block_size)

    def _full(self):
        full = [0] * ((self.k + self.m) * self.k)
        self.get_full_matrix(full, self.k)
        full[self.k * self.k:] = self.make_encoding_matrix()
        return full

    def encode_partial_blocks_for_encoding(self, data_ptrs, coding_ptrs, block_size, data_idxs,
                                           parity_idxs):  # rs.cpp:44-53
        self.encode_partial_blocks_for_encoding_(self.k, self._full(), data_ptrs, coding_ptrs, block_size,
                                                 list(data_idxs), list(parity_idxs))

    def encode_partial_blocks_for_decoding(self, data_ptrs, coding_ptrs, block_size, local_survivor_idxs,
                                           survivor_idxs, failure_idxs):  # rs.cpp:55-66
        self.encode_partial_blocks_for_decoding_(self.k, self._full(), data_ptrs, coding_ptrs, block_size,
                                                 list(local_survivor_idxs), list(survivor_idxs),
                                                 list(failure_idxs))

    def check_if_decodable(self, failure_idxs):  # rs.cpp:68-76
        return self.m >= len(failure_idxs)


class EnlargedRSCode(RSCode):
    def __init__(self, k=6, m=3):  # rs.h:44-52 (x = 2, seri_num = 1 field defaults)
        super().__init__(k, m)
        self.x = 2
        self.seri_num = 1

    def init_coding_parameters(self, cp):  # rs.cpp:282-288 (local_or_column not copied)
        self.k, self.m, self.x, self.seri_num = cp.k, cp.m, cp.x, cp.seri_num

    def make_encoding_matrix(self):  # rs.cpp:290-305
        k, m = self.k, self.m
        if self.seri_num >= self.x:
            return [0] * (k * m)  # prints "Invalid argurments!" and leaves the caller's zeros
        big = J.reed_sol_vandermonde_coding_matrix(self.x * k, m)
        out = []
        for i in range(m):
            base = i * k * self.x + self.seri_num * k
            out += big[base:base + k]
        return out


# ==================================================================== LRC family (lrc.cpp)
class LocallyRepairableCode(ErasureCode):
    def __init__(self, k, l, g):  # lrc.h:17-23
        super().__init__(k, l + g)
        self.l = l
        self.g = g
        self.r = (k + l - 1) // l

    def init_coding_parameters(self, cp):  # lrc.cpp:5-12 (r is NOT recomputed)
        self.k, self.l, self.g = cp.k, cp.l, cp.g
        self.m = cp.l + cp.g
        self.local_or_column = cp.local_or_column

    def encode(self, data_ptrs, coding_ptrs, block_size):  # lrc.cpp:23-30
        J.jerasure_matrix_encode(self.k, self.g + self.l, self.make_encoding_matrix(), data_ptrs, coding_ptrs,
                                 block_size)

    def decode(self, data_ptrs, coding_ptrs, block_size, erasures, failed_num):  # lrc.cpp:32-42
        if self.local_or_column:
            group_id = erasures[failed_num]
            erasures[failed_num] = -1
            return self.decode_local(data_ptrs, coding_ptrs, block_size, erasures, failed_num, group_id)
        return self.decode_global(data_ptrs, coding_ptrs, block_size, erasures, failed_num)

    def decode_global(self, data_ptrs, coding_ptrs, block_size, erasures, failed_num):  # lrc.cpp:44-56
        return J.jerasure_matrix_decode(self.k, self.g + self.l, self.make_encoding_matrix(), failed_num,
                                        erasures, data_ptrs, coding_ptrs, block_size)

    def decode_local(self, data_ptrs, coding_ptrs, block_size, erasures, failed_num, group_id):  # :58-72
        group_size, _min = self.get_group_size(group_id)
        gm = self.make_group_matrix(group_id, group_size)
        return J.jerasure_matrix_decode(group_size, 1, gm, failed_num, erasures, data_ptrs, coding_ptrs,
                                        block_size)

    def encode_partial_blocks_for_encoding(self, data_ptrs, coding_ptrs, block_size, data_idxs, parity_idxs):
        if self.local_or_column:  # lrc.cpp:74-85
            self.encode_partial_blocks_for_encoding_local(data_ptrs, coding_ptrs, block_size, data_idxs,
                                                          parity_idxs)
        else:
            self.encode_partial_blocks_for_encoding_global(data_ptrs, coding_ptrs, block_size, data_idxs,
                                                           parity_idxs)

    def encode_partial_blocks_for_decoding(self, data_ptrs, coding_ptrs, block_size, local_survivor_idxs,
                                           survivor_idxs, failure_idxs):  # lrc.cpp:87-101
        f = (self.encode_partial_blocks_for_decoding_local if self.local_or_column
             else self.encode_partial_blocks_for_decoding_global)
        f(data_ptrs, coding_ptrs, block_size, list(local_survivor_idxs), list(survivor_idxs),
          list(failure_idxs))

    def _full(self):
        k = self.k
        full = [0] * ((k + self.g + self.l) * k)
        self.get_full_matrix(full, k)
        full[k * k:] = self.make_encoding_matrix()
        return full

    def encode_partial_blocks_for_encoding_global(self, data_ptrs, coding_ptrs, block_size, data_idxs,
                                                  parity_idxs):  # lrc.cpp:103-113
        self.encode_partial_blocks_for_encoding_(self.k, self._full(), data_ptrs, coding_ptrs, block_size,
                                                 list(data_idxs), list(parity_idxs))

    def encode_partial_blocks_for_decoding_global(self, data_ptrs, coding_ptrs, block_size, lsi, si, fi):
        self.encode_partial_blocks_for_decoding_(self.k, self._full(), data_ptrs, coding_ptrs, block_size,
                                                 lsi, si, fi)  # lrc.cpp:115-126

    def _group_full(self, group_size, group_id):
        gm = [0] * ((group_size + 1) * group_size)
        self.get_full_matrix(gm, group_size)
        gm[group_size * group_size:] = self.make_group_matrix(group_id, group_size)
        return gm

    def _remap_local(self, idx, group_size, min_idx):
        return group_size if idx >= self.k + self.g else idx - min_idx

    def encode_partial_blocks_for_encoding_local(self, data_ptrs, coding_ptrs, block_size, data_idxs,
                                                 parity_idxs):  # lrc.cpp:128-159
        group_id = parity_idxs[0] - self.k - self.g
        group_size, min_idx = self.get_group_size(group_id)
        d_ = [self._remap_local(i, group_size, min_idx) for i in data_idxs]
        p_ = [self._remap_local(i, group_size, min_idx) for i in parity_idxs]
        self.encode_partial_blocks_for_encoding_(group_size, self._group_full(group_size, group_id), data_ptrs,
                                                 coding_ptrs, block_size, d_, p_)

    def _local_ctx(self, survivor_idxs, failure_idxs):  # lrc.cpp:165-182
        group_size = len(survivor_idxs)
        group_id = -1
        min_idx = self.k + self.g + self.l
        for idx in list(survivor_idxs) + list(failure_idxs):
            if idx >= self.k + self.g:
                group_id = idx - self.k - self.g
            if idx < min_idx:
                min_idx = idx
        return group_size, group_id, min_idx

    def encode_partial_blocks_for_decoding_local(self, data_ptrs, coding_ptrs, block_size, lsi, si, fi):
        group_size, group_id, min_idx = self._local_ctx(si, fi)  # lrc.cpp:161-213
        si_ = [self._remap_local(i, group_size, min_idx) for i in si]
        fi_ = [self._remap_local(i, group_size, min_idx) for i in fi]
        lsi_ = [self._remap_local(i, group_size, min_idx) for i in lsi]
        self.encode_partial_blocks_for_decoding_(group_size, self._group_full(group_size, group_id), data_ptrs,
                                                 coding_ptrs, block_size, lsi_, si_, fi_)

    # subclasses: make_encoding_matrix(), make_group_matrix(group_id, size), get_group_size(group_id)


def _vand(k, m):
    return J.reed_sol_vandermonde_coding_matrix(k, m)


def _mix_local(l_matrix, G, k, g, l):
    """L · [I_k ; G] over GF(2^8): the Azure+1 / Optimal-LRC local rows (lrc.cpp:951-974, 1183-1209)."""
    dg = [0] * ((k + g) * k)
    for i in range(k):
        dg[i * k + i] = 1
    dg[k * k:] = G
    return J.jerasure_matrix_multiply(l_matrix, dg, l, k + g, k + g, k)


class Azu_LRC(LocallyRepairableCode):
    def __init__(self, k, l, g):  # lrc.h:82-87
        super().__init__(k, l, g)
        self.r = (k + l - 1) // l

    def make_encoding_matrix(self):  # lrc.cpp:622-644
        k, g, l, r = self.k, self.g, self.l, self.r
        out = [0] * (k * (g + l))
        out[:g * k] = _vand(k, g)
        for i in range(l):
            for j in range(k):
                if i * r <= j < (i + 1) * r:
                    out[(i + g) * k + j] = 1
        return out

    def make_group_matrix(self, group_id, size):  # lrc.cpp:646-656
        gm = [0] * size
        for i in range(self.l):
            if i == group_id:
                for j in range(min(self.r, self.k - i * self.r)):
                    gm[j] = 1
        return gm[:size]

    def get_group_size(self, group_id):  # lrc.cpp:693-704
        min_idx = group_id * self.r
        if group_id < self.l - 1:
            return self.r, min_idx
        if group_id == self.l - 1:
            return (self.r if self.k % self.r == 0 else self.k % self.r), min_idx
        return self.g, self.k

    def bid2gid(self, b):  # lrc.cpp:665-676
        if b < self.k:
            return b // self.r
        if b < self.k + self.g:
            return self.l
        return b - self.k - self.g

    def idxingroup(self, b):  # lrc.cpp:678-691
        k, g, r, l = self.k, self.g, self.r, self.l
        if b < k:
            return b % r
        if b < k + g:
            return b - k
        if b - k - g < l - 1:
            return r
        return r if k % r == 0 else k % r


class Azu_LRC_1(LocallyRepairableCode):
    def __init__(self, k, l, g):  # lrc.h:113-118
        super().__init__(k, l, g)
        self.r = (k + l - 2) // (l - 1)

    def make_encoding_matrix(self):  # lrc.cpp:933-981
        k, g, l, r = self.k, self.g, self.l, self.r
        G = _vand(k, g)
        out = [0] * (k * (g + l))
        out[:g * k] = G
        L = [0] * (l * (k + g))
        idx = 0
        for i in range(l - 1):
            for _ in range(min(r, k - i * r)):
                L[i * (k + g) + idx] = 1
                idx += 1
        for _ in range(g):
            L[(l - 1) * (k + g) + idx] = 1
            idx += 1
        out[g * k:] = _mix_local(L, G, k, g, l)
        return out

    def make_group_matrix(self, group_id, size):  # lrc.cpp:983-999
        gm = [0] * max(size, self.g, self.r)
        if group_id == self.l - 1:
            for j in range(self.g):
                gm[j] = 1
            return gm[:size]
        for i in range(self.l - 1):
            if i == group_id:
                for j in range(min(self.r, self.k - i * self.r)):
                    gm[j] = 1
        return gm[:size]

    def get_group_size(self, group_id):  # lrc.cpp:1038-1049
        min_idx = group_id * self.r
        if group_id < self.l - 2:
            return self.r, min_idx
        if group_id == self.l - 2:
            return (self.r if self.k % self.r == 0 else self.k % self.r), min_idx
        return self.g, self.k


class Opt_LRC(LocallyRepairableCode):
    def __init__(self, k, l, g):  # lrc.h:141-146
        super().__init__(k, l, g)
        self.r = (k + g + l - 1) // l

    def make_encoding_matrix(self):  # lrc.cpp:1168-1215
        k, g, l, r = self.k, self.g, self.l, self.r
        G = _vand(k, g)
        out = [0] * (k * (g + l))
        out[:g * k] = G
        L = [0] * (l * (k + g))
        idx = 0
        for i in range(l):
            for _ in range(min(r, k + g - i * r)):
                L[i * (k + g) + idx] = 1
                idx += 1
        out[g * k:] = _mix_local(L, G, k, g, l)
        return out

    def make_group_matrix(self, group_id, size):  # lrc.cpp:1217-1227
        gm = [0] * max(size, self.r)
        for i in range(self.l):
            if i == group_id:
                for j in range(min(self.r, self.k + self.g - i * self.r)):
                    gm[j] = 1
        return gm[:size]

    def get_group_size(self, group_id):  # lrc.cpp:1260-1268
        min_idx = group_id * self.r
        if group_id < self.l - 1:
            return self.r, min_idx
        kg = self.k + self.g
        return (self.r if kg % self.r == 0 else kg % self.r), min_idx


class Opt_Cau_LRC(LocallyRepairableCode):
    def __init__(self, k, l, g):  # lrc.h:169-174
        super().__init__(k, l, g)
        self.r = (k + l - 1) // l

    def make_encoding_matrix(self):  # lrc.cpp:1485-1518
        k, g, l, r = self.k, self.g, self.l, self.r
        C = _cauchy(k, g + 1)
        out = [0] * (k * (g + l))
        out[:g * k] = C[:g * k]
        d = 0
        for i in range(l):
            for j in range(k):
                if i * r <= j < (i + 1) * r:
                    out[(i + g) * k + j] = C[g * k + d]
                    d += 1
        for i in range(l):
            for j in range(g):
                for t in range(k):  # galois_region_xor on the int rows (lrc.cpp:1509-1513)
                    out[(i + g) * k + t] ^= C[j * k + t]
        return out

    def make_group_matrix(self, group_id, size):  # lrc.cpp:1574-1591
        C = _cauchy(self.k, self.g + 1)
        gm = [0] * max(size, self.r + self.g)
        idx = 0
        for i in range(self.l):
            gs = min(self.r, self.k - i * self.r)
            for j in range(gs):
                if i == group_id:
                    gm[j] = C[self.g * self.k + idx]
                idx += 1
            for j in range(gs, gs + self.g):
                if i == group_id:
                    gm[j] = 1
        return gm[:size]

    def get_group_size(self, group_id):  # lrc.cpp:1628-1639
        min_idx = group_id * self.r
        if group_id < self.l - 1:
            return self.r + self.g, min_idx
        if group_id == self.l - 1:
            return (self.r if self.k % self.r == 0 else self.k % self.r) + self.g, min_idx
        return self.g, self.k

    def _remap_cau(self, idx, group_size, min_idx):  # lrc.cpp:1320-1340
        k, g = self.k, self.g
        if idx >= k + g:
            return group_size
        if idx >= k:
            return group_size - g + idx - k
        return idx - min_idx

    def encode_partial_blocks_for_encoding_local(self, data_ptrs, coding_ptrs, block_size, data_idxs,
                                                 parity_idxs):  # lrc.cpp:1309-1346
        group_id = parity_idxs[0] - self.k - self.g
        group_size, min_idx = self.get_group_size(group_id)
        d_ = [self._remap_cau(i, group_size, min_idx) for i in data_idxs]
        p_ = [self._remap_cau(i, group_size, min_idx) for i in parity_idxs]
        self.encode_partial_blocks_for_encoding_(group_size, self._group_full(group_size, group_id), data_ptrs,
                                                 coding_ptrs, block_size, d_, p_)

    def encode_partial_blocks_for_decoding_local(self, data_ptrs, coding_ptrs, block_size, lsi, si, fi):
        group_size, group_id, min_idx = self._local_ctx(si, fi)  # lrc.cpp:1348-1413
        si_ = [self._remap_cau(i, group_size, min_idx) for i in si]
        fi_ = [self._remap_cau(i, group_size, min_idx) for i in fi]
        lsi_ = [self._remap_cau(i, group_size, min_idx) for i in lsi]
        self.encode_partial_blocks_for_decoding_(group_size, self._group_full(group_size, group_id), data_ptrs,
                                                 coding_ptrs, block_size, lsi_, si_, fi_)


class Uni_Cau_LRC(LocallyRepairableCode):
    def __init__(self, k, l, g):  # lrc.h:212-217
        super().__init__(k, l, g)
        self.r = (k + g + l - 1) // l

    def make_encoding_matrix(self):  # lrc.cpp:2097-2156
        k, g, l, r = self.k, self.g, self.l, self.r
        C = _cauchy(k, g + 1)
        out = [0] * (k * (g + l))
        out[:g * k] = C[:g * k]
        L = [0] * (l * k)
        d = 0
        l_idx = 0
        i = 0
        while i < l and d < k:
            gs = min(r, k + g - i * r)
            j = 0
            while j < gs and d < k:
                L[i * k + d] = C[g * k + d]
                d += 1
                j += 1
            l_idx = i
            i += 1
        g_idx = 0
        for i in range(l_idx, l):
            gs = min(r, k + g - i * r)
            sub = (g - g_idx) if gs < r else (i + 1) * r - (k + g_idx)
            rows = []
            for _ in range(sub):
                rows.append(C[g_idx * k:(g_idx + 1) * k])
                g_idx += 1
            for row in rows:
                for t in range(k):
                    L[i * k + t] ^= row[t]
        out[g * k:] = L
        return out

    def make_group_matrix(self, group_id, size):  # lrc.cpp:2213-2230
        C = _cauchy(self.k, self.g + 1)
        gm = [0] * max(size, self.r)
        idx = 0
        for i in range(self.l):
            gs = min(self.r, self.k + self.g - i * self.r)
            for j in range(gs):
                if i == group_id:
                    gm[j] = C[self.g * self.k + idx] if idx < self.k else 1
                idx += 1
        return gm[:size]

    def get_group_size(self, group_id):  # lrc.cpp:2263-2271
        min_idx = group_id * self.r
        if group_id < self.l - 1:
            return self.r, min_idx
        kg = self.k + self.g
        return (self.r if kg % self.r == 0 else kg % self.r), min_idx


# ==================================================================== Product codes (pc.cpp)
class ProductCode(ErasureCode):
    def __init__(self, k1, m1, k2, m2):  # pc.h:21-24
        super().__init__(k1 * k2, (k1 + m1) * (k2 + m2) - k1 * k2)
        self.k1, self.m1, self.k2, self.m2 = k1, m1, k2, m2
        self.row_code = RSCode(k1, m1)
        self.col_code = RSCode(k2, m2)

    def init_coding_parameters(self, cp):  # pc.cpp:5-18
        self.k1, self.m1, self.k2, self.m2 = cp.k1, cp.m1, cp.k2, cp.m2
        self.k = cp.k1 * cp.k2
        self.m = (cp.k1 + cp.m1) * (cp.k2 + cp.m2) - self.k
        self.row_code.k, self.row_code.m = cp.k1, cp.m1
        self.col_code.k, self.col_code.m = cp.k2, cp.m2
        self.local_or_column = cp.local_or_column

    # codes actually used for rows / columns (HPC overrides)
    def _rowc(self):
        return self.row_code

    def _colc(self):
        return self.col_code

    def encode(self, data_ptrs, coding_ptrs, block_size):  # pc.cpp:39-76
        k1, m1, k2, m2 = self.k1, self.m1, self.k2, self.m2
        for i in range(k2):
            self._rowc().encode(data_ptrs[i * k1:(i + 1) * k1], [coding_ptrs[i * m1 + j] for j in range(m1)],
                                block_size)
        for i in range(k1 + m1):
            if i < k1:
                data = [data_ptrs[j * k1 + i] for j in range(k2)]
                coding = [coding_ptrs[k2 * m1 + j * k1 + i] for j in range(m2)]
            else:
                data = [coding_ptrs[j * m1 + i - k1] for j in range(k2)]
                coding = [coding_ptrs[k2 * m1 + k1 * m2 + j * m1 + i - k1] for j in range(m2)]
            self._colc().encode(data, coding, block_size)

    def _blocks_map(self, data_ptrs, coding_ptrs, with_global=True):
        k1, m1, k2, m2 = self.k1, self.m1, self.k2, self.m2
        bm = [[None] * (k1 + m1) for _ in range(k2 + m2)]
        di = pi = 0
        for i in range(k2):
            for j in range(k1 + m1):
                if j < k1:
                    bm[i][j] = data_ptrs[di]; di += 1
                else:
                    bm[i][j] = coding_ptrs[pi]; pi += 1
        gi = k2 * m1 + m2 * k1
        for i in range(k2, k2 + m2):
            for j in range(k1 + m1):
                if j < k1:
                    bm[i][j] = coding_ptrs[pi]; pi += 1
                elif with_global:
                    bm[i][j] = coding_ptrs[gi]; gi += 1
        return bm

    def _iterative_decode(self, bm, block_size, erasures, failed_num, ncols, nrows):
        """pc.cpp:79-195 / 890-1029 control flow: columns (≤ m2 losses) then rows (≤ m1) until done."""
        k1, m1, k2, m2 = self.k1, self.m1, self.k2, self.m2
        fmap = [[0] * (k1 + m1) for _ in range(k2 + m2)]
        frc = [0] * (k2 + m2)
        fcc = [0] * (k1 + m1)
        for i in range(failed_num):
            r, c = self.bid2rowcol(erasures[i])
            fmap[r][c] = 1
            frc[r] += 1
            fcc[c] += 1
        while failed_num > 0:
            for i in range(ncols):
                if 0 < fcc[i] <= m2:
                    er = [jj for jj in range(k2) if fmap[jj][i]] + [jj + k2 for jj in range(m2) if fmap[jj + k2][i]]
                    cnt = fcc[i]
                    self._colc().decode([bm[jj][i] for jj in range(k2)], [bm[jj + k2][i] for jj in range(m2)],
                                        block_size, er + [-1], cnt)
                    for jj in range(k2 + m2):
                        if fmap[jj][i]:
                            fmap[jj][i] = 0; failed_num -= 1; frc[jj] -= 1; fcc[i] -= 1
            if failed_num == 0:
                break
            max_row = -1
            for i in range(nrows):
                if 0 < frc[i] <= m1:
                    max_row = i
                    er = [jj for jj in range(k1) if fmap[i][jj]] + [jj + k1 for jj in range(m1) if fmap[i][jj + k1]]
                    cnt = frc[i]
                    self._rowc().decode([bm[i][jj] for jj in range(k1)], [bm[i][jj + k1] for jj in range(m1)],
                                        block_size, er + [-1], cnt)
                    for jj in range(k1 + m1):
                        if fmap[i][jj]:
                            fmap[i][jj] = 0; failed_num -= 1; frc[i] -= 1; fcc[jj] -= 1
            if max_row == -1:
                return -1
        return 0

    def decode(self, data_ptrs, coding_ptrs, block_size, erasures, failed_num):  # pc.cpp:79-195
        bm = self._blocks_map(data_ptrs, coding_ptrs)
        return self._iterative_decode(bm, block_size, erasures, failed_num, self.k1 + self.m1, self.k2 + self.m2)

    def _map_idxs(self, idxs, use_row):
        out = []
        for b in idxs:
            r, c = self.bid2rowcol(b)
            out.append(r if use_row else c)
        return out

    def _partial_codes(self):
        return self.col_code, self.row_code

    def encode_partial_blocks_for_encoding(self, data_ptrs, coding_ptrs, block_size, data_idxs,
                                           parity_idxs):  # pc.cpp:257-288
        colc, rowc = self._partial_codes()
        use_row = self.local_or_column
        code = colc if use_row else rowc
        code.encode_partial_blocks_for_encoding(data_ptrs, coding_ptrs, block_size,
                                                self._map_idxs(data_idxs, use_row),
                                                self._map_idxs(parity_idxs, use_row))

    def encode_partial_blocks_for_decoding(self, data_ptrs, coding_ptrs, block_size, lsi, si, fi):
        colc, rowc = self._partial_codes()  # pc.cpp:290-324
        use_row = self.local_or_column
        code = colc if use_row else rowc
        code.encode_partial_blocks_for_decoding(data_ptrs, coding_ptrs, block_size, self._map_idxs(lsi, use_row),
                                                self._map_idxs(si, use_row), self._map_idxs(fi, use_row))

    def rowcol2bid(self, row, col):  # pc.cpp:326-340
        k1, m1, k2, m2 = self.k1, self.m1, self.k2, self.m2
        if row < k2 and col < k1:
            return row * k1 + col
        if row < k2:
            return k1 * k2 + row * m1 + (col - k1)
        if col < k1:
            return (k1 + m1) * k2 + (row - k2) * k1 + col
        return (k1 + m1) * k2 + k1 * m2 + (row - k2) * m1 + (col - k1)

    def bid2rowcol(self, bid):  # pc.cpp:342-359
        k1, m1, k2, m2 = self.k1, self.m1, self.k2, self.m2
        if bid < k1 * k2:
            return bid // k1, bid % k1
        if bid < (k1 + m1) * k2:
            t = bid - k1 * k2
            return t // m1, t % m1 + k1
        if bid < (k1 + m1) * k2 + k1 * m2:
            t = bid - (k1 + m1) * k2
            return t // k1 + k2, t % k1
        t = bid - (k1 + m1) * k2 - k1 * m2
        return t // m1 + k2, t % m1 + k1


class HPC(ProductCode):
    def __init__(self, k1, m1, k2, m2):  # pc.h:69-72
        super().__init__(k1, m1, k2, m2)
        self.e_row_code = EnlargedRSCode(k1, m1)
        self.e_col_code = EnlargedRSCode(k2, m2)
        self.isvertical = True

    def init_coding_parameters(self, cp):  # pc.cpp:553-574
        super().init_coding_parameters(cp)
        for c, (kk, mm) in ((self.e_row_code, (cp.k1, cp.m1)), (self.e_col_code, (cp.k2, cp.m2))):
            c.k, c.m, c.x, c.seri_num = kk, mm, cp.x, cp.seri_num

    def _rowc(self):  # pc.cpp:585-589, 718-724
        return self.row_code if self.isvertical else self.e_row_code

    def _colc(self):  # pc.cpp:613-619, 680-686
        return self.e_col_code if self.isvertical else self.col_code

    def _partial_codes(self):  # pc.cpp:755-835
        if self.isvertical:
            return self.e_col_code, self.row_code
        return self.col_code, self.e_row_code


class HVPC(ProductCode):
    def __init__(self, k1, m1, k2, m2):  # pc.h:101-106
        super().__init__(k1, m1, k2, m2)
        self.m = k1 * m2 + k2 * m1

    def init_coding_parameters(self, cp):  # pc.cpp:869-882
        super().init_coding_parameters(cp)
        self.m = cp.k1 * cp.m2 + cp.k2 * cp.m1

    def encode(self, data_ptrs, coding_ptrs, block_size):  # pc.cpp:890-918
        k1, m1, k2, m2 = self.k1, self.m1, self.k2, self.m2
        for i in range(k2):
            self.row_code.encode(data_ptrs[i * k1:(i + 1) * k1], [coding_ptrs[i * m1 + j] for j in range(m1)],
                                 block_size)
        for i in range(k1):
            self.col_code.encode([data_ptrs[j * k1 + i] for j in range(k2)],
                                 [coding_ptrs[k2 * m1 + j * k1 + i] for j in range(m2)], block_size)

    def decode(self, data_ptrs, coding_ptrs, block_size, erasures, failed_num):  # pc.cpp:921-1029
        bm = self._blocks_map(data_ptrs, coding_ptrs, with_global=False)
        return self._iterative_decode(bm, block_size, erasures, failed_num, self.k1, self.k2)


def ec_factory(ec_type, cp: CodingParameters):  # metadata.cpp:48-77
    t = ECTYPE(ec_type)
    if t == ECTYPE.RS:
        return RSCode(cp.k, cp.m)
    if t == ECTYPE.ERS:
        ec = EnlargedRSCode(cp.k, cp.m)
        ec.init_coding_parameters(cp)
        return ec
    if t == ECTYPE.AZURE_LRC:
        return Azu_LRC(cp.k, cp.l, cp.g)
    if t == ECTYPE.AZURE_LRC_1:
        return Azu_LRC_1(cp.k, cp.l, cp.g)
    if t == ECTYPE.OPTIMAL_LRC:
        return Opt_LRC(cp.k, cp.l, cp.g)
    if t == ECTYPE.OPTIMAL_CAUCHY_LRC:
        return Opt_Cau_LRC(cp.k, cp.l, cp.g)
    if t == ECTYPE.UNIFORM_CAUCHY_LRC:
        return Uni_Cau_LRC(cp.k, cp.l, cp.g)
    if t == ECTYPE.PC:
        return ProductCode(cp.k1, cp.m1, cp.k2, cp.m2)
    if t == ECTYPE.Hierachical_PC:
        ec = HPC(cp.k1, cp.m1, cp.k2, cp.m2)
        ec.init_coding_parameters(cp)
        return ec
    if t == ECTYPE.HV_PC:
        return HVPC(cp.k1, cp.m1, cp.k2, cp.m2)
    return None


def blocks(n, size, seed=0):
    """n fresh B-byte buffers of splitmix bytes (helper for tests)."""
    return [J.splitmix_bytes(seed, i * ((size + 7) // 8), size) for i in range(n)]


def zeros(n, size):
    return [np.zeros(size, dtype=np.uint8) for _ in range(n)]
