"""Pin the ORACLE (oracle/jerasure_w8.c + oracle/ec_ref.py) before trusting it (CPU only).

Parity status: the real Jerasure / gf-complete are absent from /root/reference and from this image
(install_third_party.sh:36,49 git-clones unpinned HEADs), the reference ships no golden vectors and its
byte-level tests are commented out.  So the oracle is pinned by:
  * published GF(2^8)/0x11d known answers (the antilog table of generator 2, inverses);
  * the structural invariants the reference relies on (Vandermonde row 0 / column 0 all ones, which
    makes jerasure_matrix_decode's row_k_ones shortcut at rs.cpp:36 correct; MDS);
  * the property tests the reference wrote but commented out (test_rs.cpp:63-326,
    test_lrc.cpp:359-593, test_pc.cpp:54-56), made deterministic;
  * the committed golden fixtures (tests/golden/golden.json, regression pin).
"""
import itertools
import json
import os
import random

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

# Antilog table of generator 2 in GF(2^8) with x^8+x^4+x^3+x^2+1 (0x11d): the standard table used by
# RAID-6 / QR codes / gf-complete w=8 (first 64 entries).
EXP_0x11D = [1, 2, 4, 8, 16, 32, 64, 128, 29, 58, 116, 232, 205, 135, 19, 38, 76, 152, 45, 90, 180, 117, 234,
             201, 143, 3, 6, 12, 24, 48, 96, 192, 157, 39, 78, 156, 37, 74, 148, 53, 106, 212, 181, 119, 238,
             193, 159, 35, 70, 140, 5, 10, 20, 40, 80, 160, 93, 186, 105, 210, 185, 111, 222, 161]


def test_field_known_answers(oracle):
    x = 1
    for i, e in enumerate(EXP_0x11D):
        assert x == e, i
        x = oracle.galois_single_multiply(x, 2)
    # generator 2 has order 255
    x, order = 2, 1
    while x != 1:
        x = oracle.galois_single_multiply(x, 2)
        order += 1
    assert order == 255
    assert oracle.galois_single_divide(1, 2) == 142  # 2^-1 = 0x8e under 0x11d
    assert oracle.galois_single_divide(0, 7) == 0
    assert oracle.galois_single_divide(5, 0) == -1  # Jerasure 2.0 convention
    for a in range(1, 256):
        assert oracle.galois_single_multiply(a, oracle.galois_single_divide(1, a)) == 1


def _is_invertible(oracle, rows, k):
    flat = [v for r in rows for v in r]
    rc, _ = oracle.jerasure_invert_matrix(flat, k)
    return rc == 0


@pytest.mark.parametrize("k,m", [(6, 2), (6, 4), (10, 4), (12, 2), (8, 1), (4, 1), (12, 4), (8, 3)])
def test_vandermonde_structure_and_mds(oracle, k, m):
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    rows = [M[i * k:(i + 1) * k] for i in range(m)]
    assert rows[0] == [1] * k                      # row k of the distribution matrix is all ones
    assert all(r[0] == 1 for r in rows)            # column 0 of the coding rows is all ones
    full = [[int(i == j) for j in range(k)] for i in range(k)] + rows
    for subset in itertools.combinations(range(k + m), k):  # every k x k submatrix of [I;M] invertible
        assert _is_invertible(oracle, [full[i] for i in subset], k), subset


def test_rs10_4_matches_survey_restatement(oracle):
    # candidate RS(10,4) coding matrix from an independent restatement of A.2.
    M = oracle.reed_sol_vandermonde_coding_matrix(10, 4)
    assert M == [1] * 10 + [1, 147, 138, 73, 93, 161, 103, 58, 99, 178] + \
        [1, 103, 156, 151, 123, 187, 166, 175, 244, 83] + [1, 220, 166, 123, 82, 143, 245, 40, 167, 122]


def _clmul_11d(a, b):
    """GF(2^8)/0x11d product by shift-and-add (no tables): independent of the oracle's field code."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
    return r


def _closed_form_vandermonde(k, m):
    """The systematic Vandermonde coding matrix from its closed form, by a route that shares no step with
    the oracle's column elimination (oracle/jerasure_w8.c:121-169):
      * V = the (k+m) x k extended Vandermonde matrix: row 0 = e_0 (point 0), row k+m-1 = e_{k-1} (the point
        at infinity), row i = (1, i, i^2, ...) in between (Plank & Ding, "Note: Correction to the 1997
        tutorial on Reed-Solomon coding", 2005; Jerasure 2.0 reed_sol_extended_vandermonde_matrix);
      * the systematic form is V * inv(V_top): the top k x k is invertible (distinct points) and every leading
        minor of V_top is a Vandermonde minor, so the library's column elimination reaches it with no swap;
      * then the library's two normalisations (reed_sol_big_vandermonde_distribution_matrix): each column
        of the coding rows divided by its entry in coding row 0, then each coding row divided by its column-0
        entry.
    The inverse is Gauss-Jordan over GF(2^8) with row pivoting, written here from scratch."""
    n = k + m
    mul = _clmul_11d
    inv_tab = [0] * 256
    for a in range(1, 256):
        inv_tab[a] = next(b for b in range(1, 256) if mul(a, b) == 1)

    def row(i):
        if i == 0:
            return [1] + [0] * (k - 1)
        if i == n - 1 and n > 1:
            return [0] * (k - 1) + [1]
        out, x = [], 1
        for _ in range(k):
            out.append(x)
            x = mul(x, i)
        return out

    V = [row(i) for i in range(n)]
    A = [r[:] + [int(i == j) for j in range(k)] for i, r in enumerate(V[:k])]
    for c in range(k):
        p = next(r for r in range(c, k) if A[r][c])
        A[c], A[p] = A[p], A[c]
        s = inv_tab[A[c][c]]
        A[c] = [mul(s, x) for x in A[c]]
        for r in range(k):
            if r != c and A[r][c]:
                f = A[r][c]
                A[r] = [x ^ mul(f, y) for x, y in zip(A[r], A[c])]
    inv_top = [r[k:] for r in A]
    C = [[0] * k for _ in range(m)]
    for i in range(m):
        for j in range(k):
            acc = 0
            for t in range(k):
                acc ^= mul(V[k + i][t], inv_top[t][j])
            C[i][j] = acc
    for j in range(k):
        s = inv_tab[C[0][j]]
        for i in range(m):
            C[i][j] = mul(C[i][j], s)
    for i in range(1, m):
        s = inv_tab[C[i][0]]
        C[i] = [mul(x, s) for x in C[i]]
    return [x for r in C for x in r]


@pytest.mark.parametrize("k,m", [(k, m) for k in range(1, 17) for m in range(1, 7)] +
                         [(10, 4), (12, 4), (20, 4), (24, 8), (40, 16), (64, 8), (100, 4)])
def test_vandermonde_matches_closed_form(oracle, k, m):
    assert oracle.reed_sol_vandermonde_coding_matrix(k, m) == _closed_form_vandermonde(k, m)


def test_cauchy(oracle):
    assert oracle.cauchy_n_ones(1) == 8
    assert oracle.cauchy_n_ones(2) == 11  # columns 2,4,..,128,29: seven single bits + popcount(0x1d)=4
    k, m = 8, 3
    orig = oracle.cauchy_original_coding_matrix(k, m)
    for i in range(m):
        for j in range(k):
            assert oracle.galois_single_multiply(orig[i * k + j], i ^ (m + j)) == 1
    C = oracle.cauchy_good_general_coding_matrix(k, m)
    assert C[:k] == [1] * k
    full = [[int(i == j) for j in range(k)] for i in range(k)] + [C[i * k:(i + 1) * k] for i in range(m)]
    for subset in itertools.combinations(range(k + m), k):
        assert _is_invertible(oracle, [full[i] for i in subset], k)
    # the improvement never increases the bit-matrix ones of a row
    for i in range(1, m):
        scaled = sum(oracle.cauchy_n_ones(v) for v in C[i * k:(i + 1) * k])
        col_norm = [oracle.galois_single_multiply(orig[i * k + j], oracle.galois_single_divide(1, orig[j]))
                    for j in range(k)]
        assert scaled <= sum(oracle.cauchy_n_ones(v) for v in col_norm)
    assert oracle.cauchy_good_general_coding_matrix(8, 2) is None  # cbest_8: unpinned, refused


def test_invert_and_multiply(oracle):
    rng = random.Random(7)
    for n in (1, 2, 5, 10, 16):
        while True:
            A = [rng.randrange(256) for _ in range(n * n)]
            rc, inv = oracle.jerasure_invert_matrix(list(A), n)
            if rc == 0:
                break
        P = oracle.jerasure_matrix_multiply(A, inv, n, n, n, n)
        assert P == [int(i == j) for i in range(n) for j in range(n)]
    rc, _ = oracle.jerasure_invert_matrix([1, 2, 2, 4], 2)  # row 2 = 2 * row 1
    assert rc == -1


def test_golden_regression(oracle):
    from oracle import ec_ref as E
    g = json.load(open(os.path.join(HERE, "golden", "golden.json")))
    B = g["block_size"]
    for c in g["codes"]:
        ec = E.ec_factory(c["type"], E.CodingParameters(**c["params"]))
        if "matrix" in c:
            assert ec.make_encoding_matrix() == c["matrix"], c["name"]
        data = [np.frombuffer(bytes.fromhex(h), dtype=np.uint8).copy() for h in c["data_hex"]]
        coding = E.zeros(ec.m, B)
        ec.encode(data, coding, B)
        assert [x.tobytes().hex() for x in coding] == c["coding_hex"], c["name"]


def test_simd_baseline_matches_scalar(oracle):
    k, m, B = 10, 4, 4096 + 37
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    data = [oracle.splitmix_bytes(3, i * 1000, B) for i in range(k)]
    a = [np.zeros(B, np.uint8) for _ in range(m)]
    b = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data, a, B)
    oracle.jerasure_matrix_encode_simd(k, m, M, data, b, B)
    assert all((x == y).all() for x, y in zip(a, b))
    S = 5
    flat = np.concatenate(data * S)
    out = np.zeros(S * m * B, np.uint8)
    assert oracle.encode_batch_mt(k, m, M, flat, out, B, S, 3) > 0
    for s in range(S):
        for i in range(m):
            assert (out[(s * m + i) * B:(s * m + i + 1) * B] == a[i]).all()



def test_call_sequence_baseline_matches_call_by_call(oracle):
    """bench.py's config3 / config4 CPU baselines (ref.call_seq_batch_mt): a per-stripe sequence of
    jerasure_matrix_encode(kin, 1) calls through scratch blocks, several threads, equals the same calls made
    one by one -- here a partial-decoding repair (two partials + perform_addition) and a GENERAL row."""
    S, nb, B = 9, 8, 1000 + 13
    stripes = oracle.splitmix_bytes(7, 0, S * nb * B).reshape(S, nb, B)
    out = np.zeros((S, 2, B), np.uint8)
    pats = [[(nb + 2, [0, 1, 2], [1, 1, 1]), (nb + 3, [3, 4, 5], [7, 1, 9]), (nb, [nb + 2, nb + 3], [1, 1])],
            [(nb + 1, [6, 7, 0], [3, 200, 1]), (nb, [nb + 1], [1])]]
    pat = np.arange(S) % 2
    assert oracle.call_seq_batch_mt(stripes, out, pats, pat, 2, 4) > 0
    for s in range(S):
        blocks = [stripes[s, j].copy() for j in range(nb)] + [np.zeros(B, np.uint8) for _ in range(4)]
        for dst, src, coef in pats[pat[s]]:
            res = [np.zeros(B, np.uint8)]
            oracle.jerasure_matrix_encode(len(src), 1, coef, [blocks[i] for i in src], res, B)
            blocks[dst] = res[0]
        assert np.array_equal(out[s, 0], blocks[nb]), s

def test_pc_merge_plan_is_the_proxies_row_sequence(oracle):
    """bench.py's pc_merge_plan (the calls ecg_replay_merge and config 4's CPU baseline issue): the helper's
    block ids map through PC(8,1,4,1)'s bid2rowcol (pc.cpp:342-359) to columns 4..7 of their row and the
    parity id to that row's parity column; run through the oracle -- the helper's partial with a PC(8,1,4,1)
    handle (pc.cpp:257-285), the main partial with an RS(8,1) handle, their XOR (perform_addition) -- every
    merged row parity equals the XOR of the row's 8 blocks of the two old stripes."""
    import sys
    sys.argv = sys.argv[:1]
    import bench
    from oracle import ec_ref as E
    mb, mc, mp, hb, hi, hp = bench.pc_merge_plan(25)
    pc = E.ec_factory(E.ECTYPE.PC, E.CodingParameters(k1=8, m1=1, k2=4, m2=1))
    pc.init_coding_parameters(E.CodingParameters(k1=8, m1=1, k2=4, m2=1))
    rs = E.RSCode(8, 1)
    old = E.ec_factory(E.ECTYPE.PC, E.CodingParameters(k1=4, m1=1, k2=4, m2=1))
    old.init_coding_parameters(E.CodingParameters(k1=4, m1=1, k2=4, m2=1))
    B = 64 + 5
    blocks = [b for b in E.blocks(50, B, 21)]
    for row in range(5):
        assert [pc.bid2rowcol(int(i)) for i in hi[row]] == [(row, 4 + c) for c in range(4)]
        assert pc.bid2rowcol(int(hp[row])) == (row, 8)
        assert [old.bid2rowcol(int(b)) for b in mb[row]] == [(row, c) for c in range(4)]
        assert [old.bid2rowcol(int(b) - 25) for b in hb[row]] == [(row, c) for c in range(4)]
        assert list(mc[row]) == [0, 1, 2, 3] and mp[row] == 8
        p0, p1 = E.zeros(1, B), E.zeros(1, B)
        pc.encode_partial_blocks_for_encoding([blocks[b] for b in hb[row]], p0, B, [int(i) for i in hi[row]],
                                              [int(hp[row])])
        rs.encode_partial_blocks_for_encoding([blocks[b] for b in mb[row]], p1, B, [int(i) for i in mc[row]],
                                              [int(mp[row])])
        want = np.bitwise_xor.reduce(np.stack([blocks[b] for b in list(mb[row]) + list(hb[row])]), axis=0)
        assert np.array_equal(p0[0] ^ p1[0], want), row


# ------------------------------------------------------------- reference property tests, made live

def _stripe(ec, B, seed):
    from oracle import ec_ref as E
    data = E.blocks(ec.k, B, seed)
    coding = E.zeros(ec.m, B)
    ec.encode(data, coding, B)
    return data + coding


@pytest.mark.parametrize("k,m", [(6, 2), (6, 4), (10, 4), (8, 1)])
def test_rs_decode_all_patterns(oracle, k, m):
    """test_rs.cpp:63-106 for every erasure pattern of size 1..m."""
    from oracle import ec_ref as E
    B = 48
    ec = E.RSCode(k, m)
    stripe = _stripe(ec, B, 11)
    for f in range(1, m + 1):
        for pat in itertools.combinations(range(k + m), f):
            blocks = [b.copy() for b in stripe]
            for i in pat:
                blocks[i][:] = 0
            assert ec.decode(blocks[:k], blocks[k:], B, list(pat) + [-1], f) == 0
            assert all((blocks[i] == stripe[i]).all() for i in range(k + m)), pat


def _partial_decode_check(ec, stripe, B, failures, survivors, split):
    """test_rs.cpp:108-225: XOR of the two partial-decoding outputs == the lost blocks."""
    from oracle import ec_ref as E
    f = len(failures)
    l1, l2 = survivors[:split], survivors[split:]
    part = E.zeros(2 * f, B)
    ec.encode_partial_blocks_for_decoding([stripe[i] for i in l1], part[:f], B, l1, survivors, failures)
    ec.encode_partial_blocks_for_decoding([stripe[i] for i in l2], part[f:], B, l2, survivors, failures)
    rep = E.zeros(f, B)
    ec.perform_addition(part, rep, B, 2 * f, f)
    return all((rep[i] == stripe[failures[i]]).all() for i in range(f))


def _partial_encode_check(ec, stripe, B, d1, d2, parity):
    """test_rs.cpp:227-326: XOR of the two partial-encoding outputs == the parities."""
    from oracle import ec_ref as E
    p = len(parity)
    part = E.zeros(2 * p, B)
    ec.encode_partial_blocks_for_encoding([stripe[i] for i in d1], part[:p], B, d1, parity)
    ec.encode_partial_blocks_for_encoding([stripe[i] for i in d2], part[p:], B, d2, parity)
    out = E.zeros(p, B)
    ec.perform_addition(part, out, B, 2 * p, p)
    return all((out[i] == stripe[parity[i]]).all() for i in range(p))


@pytest.mark.parametrize("k,m", [(6, 2), (10, 4), (12, 4)])
def test_rs_partial_properties(oracle, k, m):
    from oracle import ec_ref as E
    rng = random.Random(k * 100 + m)
    B = 32
    ec = E.RSCode(k, m)
    stripe = _stripe(ec, B, 5)
    for _ in range(20):
        f = rng.randint(1, m)
        failures = rng.sample(range(k + m), f)
        survivors = rng.sample([i for i in range(k + m) if i not in failures], k)
        assert _partial_decode_check(ec, stripe, B, failures, survivors, rng.randint(1, k - 1))
        data = list(range(k))
        rng.shuffle(data)
        cut = rng.randint(1, k - 1)
        parity = list(range(k, k + m))
        rng.shuffle(parity)
        assert _partial_encode_check(ec, stripe, B, data[:cut], data[cut:], parity)


LRCS = [("AZURE_LRC", 8, 2, 2), ("AZURE_LRC", 12, 2, 2), ("AZURE_LRC_1", 8, 3, 2), ("OPTIMAL_LRC", 8, 2, 2),
        ("OPTIMAL_CAUCHY_LRC", 8, 2, 2), ("UNIFORM_CAUCHY_LRC", 8, 2, 2)]


@pytest.mark.parametrize("name,k,l,g", LRCS)
def test_lrc_global_decode_and_partials(oracle, name, k, l, g):
    """test_lrc.cpp:359-593 (global path): decode and partial coding over the full (k+g+l) x k matrix."""
    from oracle import ec_ref as E
    rng = random.Random(hash(name) & 0xffff)
    B = 32
    ec = E.ec_factory(E.ECTYPE[name], E.CodingParameters(k=k, l=l, g=g))
    stripe = _stripe(ec, B, 9)
    n = k + g + l
    ok = 0
    for f in range(1, g + 1):  # any <= g failures among data + globals are recoverable by the globals
        for pat in itertools.combinations(range(k + g), f):
            blocks = [b.copy() for b in stripe]
            for i in pat:
                blocks[i][:] = 0
            if ec.decode(blocks[:k], blocks[k:], B, list(pat) + [-1], f) == 0:
                assert all((blocks[i] == stripe[i]).all() for i in range(n)), pat
                ok += 1
    assert ok > 0
    for _ in range(10):
        failures = rng.sample(range(k + g), rng.randint(1, g))
        survivors = [i for i in range(k + g) if i not in failures][:k]
        assert _partial_decode_check(ec, stripe, B, failures, survivors, rng.randint(1, k - 1))
        data = list(range(k))
        rng.shuffle(data)
        cut = rng.randint(1, k - 1)
        parity = list(range(k, k + g))
        assert _partial_encode_check(ec, stripe, B, data[:cut], data[cut:], parity)


@pytest.mark.parametrize("name,k,l,g", [x for x in LRCS if x[0] in ("AZURE_LRC", "OPTIMAL_LRC")])
def test_lrc_local_repair(oracle, name, k, l, g):
    """Single data-block local repair inside its group (decode_local, lrc.cpp:58-72, and the partial
    local path lrc.cpp:161-213) as main_repair drives it (handle_repair.cpp:234-384)."""
    from oracle import ec_ref as E
    B = 32
    ec = E.ec_factory(E.ECTYPE[name], E.CodingParameters(k=k, l=l, g=g))
    stripe = _stripe(ec, B, 13)
    ec.local_or_column = True
    groups = []
    idx = 0
    span = k if name == "AZURE_LRC" else k + g
    for i in range(l):
        size = min(ec.r, span - i * ec.r)
        groups.append(list(range(idx, idx + size)) + [k + g + i])
        idx += size
    for gid, members in enumerate(groups):
        for lost in members[:-1]:
            surv = [b for b in members if b != lost]
            # decode_local: group-space data = members except local parity, coding = local parity
            gs, min_idx = ec.get_group_size(gid)
            data = [stripe[b].copy() for b in members[:-1]]
            coding = [stripe[members[-1]].copy()]
            pos = members.index(lost)
            data[pos][:] = 0
            er = [pos, gid]
            assert ec.decode(data, coding, B, er, 1) == 0
            assert (data[pos] == stripe[lost]).all()
            # partial local decoding, split in two helpers
            assert _partial_decode_check(ec, stripe, B, [lost], surv, len(surv) // 2)


@pytest.mark.parametrize("t", ["PC", "Hierachical_PC", "HV_PC"])
def test_product_codes_decode(oracle, t):
    """test_pc.cpp:54-56 (commented out upstream): iterative row/column decode recovers the data."""
    from oracle import ec_ref as E
    rng = random.Random(3)
    B = 32
    params = dict(k1=4, m1=2, k2=2, m2=1, x=2, seri_num=1)
    ec = E.ec_factory(E.ECTYPE[t], E.CodingParameters(**params))
    stripe = _stripe(ec, B, 21)
    n = ec.k + ec.m
    tried = 0
    for _ in range(40):
        pat = rng.sample(range(n), rng.randint(1, 3))
        blocks = [b.copy() for b in stripe]
        for i in pat:
            blocks[i][:] = 0
        rc = ec.decode(blocks[:ec.k], blocks[ec.k:], B, list(pat), len(pat))
        if rc == 0 and (t != "Hierachical_PC" or len(pat) == 1):
            assert all((blocks[i] == stripe[i]).all() for i in range(n)), pat
            tried += 1
    assert tried > 0
