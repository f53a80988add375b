"""GPU parity: the HIP path (through libecg.so's C ABI) against the oracle on the same inputs.

Bit-exact for every byte.  Small sizes are compared against the oracle directly; BASELINE.json's full
size (RS(10,4), 1 MiB blocks, 4096 stripes) is checked through size-independent properties
(encode -> erase -> decode round trips on device) plus oracle comparisons of sampled stripes.
"""
import itertools
import json
import os
import random
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    return torch


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


# ------------------------------------------------------------------ Jerasure-compatible tier (host buffers)

@pytest.mark.parametrize("k,m", [(10, 4), (6, 4), (6, 2), (12, 4), (8, 1), (1, 1), (40, 8), (130, 3)])
@pytest.mark.parametrize("B", [1, 15, 16, 64, 1000, 4099, 65536])
def test_matrix_encode_host(ecg, oracle, torch_cuda, k, m, B):
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m) if k + m <= 256 else None
    data = [rnd(B, 100 * j + B) for j in range(k)]
    a = [np.zeros(B, np.uint8) for _ in range(m)]
    b = [np.full(B, 0x5a, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data, a, B)
    ecg.jerasure_matrix_encode(k, m, M, data, b, B)
    assert same(a, b)


def test_matrix_encode_random_matrices(ecg, oracle, torch_cuda):
    """Arbitrary coefficient matrices (zeros, ones, all-zero rows left untouched)."""
    rng = random.Random(2)
    B = 777
    for trial in range(30):
        k, m = rng.randint(1, 20), rng.randint(1, 12)
        M = [rng.choice([0, 1, rng.randrange(256)]) for _ in range(k * m)]
        if trial % 5 == 0:
            M[:k] = [0] * k  # all-zero row: destination untouched
        data = [rnd(B, trial * 50 + j) for j in range(k)]
        a = [rnd(B, 999 + i) for i in range(m)]
        b = [x.copy() for x in a]
        oracle.jerasure_matrix_encode(k, m, M, data, a, B)
        ecg.jerasure_matrix_encode(k, m, M, data, b, B)
        assert same(a, b), (k, m, M)


@pytest.mark.parametrize("lat_dword", [None, 0, 1 << 20])
def test_latency_kernel_shapes(ecg, oracle, torch_cuda, lat_dword):
    """Zero-copy host calls at 16-byte multiples: the 4-bytes-per-lane latency kernel (blocks up to
    ECG_OPT_LAT_DWORD_BYTES; every input-count bucket 4/6/8/10/12/16 with padded inputs, GENERAL and
    BINARY, row tiles) and the 16-byte latency kernel above it, each call checked at once; at the
    default threshold, with the 16-byte kernel only (0) and with the 4-byte kernel only (1 MiB)."""
    saved = ecg.get_option(ecg.ECG_OPT_LAT_DWORD_BYTES)
    if lat_dword is not None:
        ecg.set_option(ecg.ECG_OPT_LAT_DWORD_BYTES, lat_dword)
    try:
        _latency_kernel_shapes(ecg, oracle)
    finally:
        ecg.set_option(ecg.ECG_OPT_LAT_DWORD_BYTES, saved)


def _latency_kernel_shapes(ecg, oracle):
    rng = random.Random(11)
    for B in (16, 1024, 4096, 16384, 16400, 32768, 32784):
        for k in range(1, 19):
            m = rng.randint(1, 9)
            kind = rng.randrange(3)
            if kind == 0:
                M = [rng.randrange(256) for _ in range(k * m)]
            elif kind == 1:
                M = [rng.randrange(2) for _ in range(k * m)]  # BINARY flavour
            else:
                M = oracle.reed_sol_vandermonde_coding_matrix(k, m) if k + m <= 256 else [1] * (k * m)
            data = [rnd(B, 7000 + 31 * k + j + B) for j in range(k)]
            a = [rnd(B, 800 + i) for i in range(m)]
            b = [x.copy() for x in a]
            oracle.jerasure_matrix_encode(k, m, M, data, a, B)
            ecg.jerasure_matrix_encode(k, m, M, data, b, B)
            assert same(a, b), (B, k, m, kind)
    for B, k, m in ((1024, 6, 32), (16384, 16, 20)):  # several row tiles, up to 32 outputs
        M = [rng.randrange(256) for _ in range(k * m)]
        data = [rnd(B, 9100 + j) for j in range(k)]
        a = [rnd(B, 9200 + i) for i in range(m)]
        b = [x.copy() for x in a]
        oracle.jerasure_matrix_encode(k, m, M, data, a, B)
        ecg.jerasure_matrix_encode(k, m, M, data, b, B)
        assert same(a, b), (B, k, m)


def test_flagged_calls_never_read_stale(ecg, oracle, torch_cuda):
    """Back-to-back host calls with fresh data every call -- RS(6,4) 1 KiB, RS(12,4) 4 KiB, RS(10,4)
    16 KiB (16 workgroups, 16 flags per output tile) encodes, every fourth followed by a decode: each
    call's output is compared before the next call (a completion flag posted before the outputs reach
    host memory shows up here as stale bytes)."""
    for k, m, B, n in ((6, 4, 1024, 2000), (12, 4, 4096, 1000), (10, 4, 16384, 300)):
        M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
        rng = np.random.default_rng(k)
        out = [np.zeros(B, np.uint8) for _ in range(m)]
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        bad = bad_dec = 0
        for i in range(n):
            data = list(rng.integers(0, 256, (k, B), dtype=np.uint8))
            ecg.jerasure_matrix_encode(k, m, M, data, out, B)
            oracle.jerasure_matrix_encode(k, m, M, data, ref, B)
            bad += not same(out, ref)
            if i % 4 == 0:  # and a decode of one lost data block, from fresh survivors
                lost = i % k
                d = [x.copy() for x in data]
                d[lost][:] = 0
                ecg.jerasure_matrix_decode(k, m, M, 1, [lost, -1], d, [x.copy() for x in ref], B)
                bad_dec += not np.array_equal(d[lost], data[lost])
        assert bad == 0 and bad_dec == 0, (k, m, B, bad, bad_dec)


@pytest.mark.parametrize("k,m,row_k_ones", [(6, 4, 1), (6, 4, 0), (10, 4, 1), (4, 2, 1)])
def test_matrix_decode_host_all_patterns(ecg, oracle, torch_cuda, k, m, row_k_ones):
    B = 1024 + 7
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    data = [rnd(B, j) for j in range(k)]
    coding = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data, coding, B)
    stripe = data + coding
    for f in range(1, m + 2):
        for pat in itertools.combinations(range(k + m), f):
            if f > 2 and k >= 10 and random.Random(hash(pat)).random() < 0.8:
                continue
            A = [x.copy() for x in stripe]
            Bb = [x.copy() for x in stripe]
            for i in pat:  # erased buffers hold garbage, not zeros
                A[i][:] = 0xEE
                Bb[i][:] = 0xEE
            ra = oracle.jerasure_matrix_decode(k, m, M, row_k_ones, list(pat) + [-1], A[:k], A[k:], B)
            rb = ecg.jerasure_matrix_decode(k, m, M, row_k_ones, list(pat) + [-1], Bb[:k], Bb[k:], B)
            assert ra == rb, pat
            assert same(A, Bb), pat
            if f <= m:
                assert ra == 0 and same(A, stripe)


def test_matrix_decode_quirky_matrices(ecg, oracle, torch_cuda):
    """Non-MDS / non-all-ones-row matrices: row_k_ones misuse (Appendix B.1) and singular patterns
    must be reproduced exactly, garbage included."""
    rng = random.Random(5)
    B = 200
    for trial in range(60):
        k, m = rng.randint(2, 8), rng.randint(1, 4)
        M = [rng.choice([0, 1, 2, rng.randrange(256)]) for _ in range(k * m)]
        stripe = [rnd(B, trial * 20 + j) for j in range(k + m)]
        pat = rng.sample(range(k + m), rng.randint(1, m))
        A = [x.copy() for x in stripe]
        Bb = [x.copy() for x in stripe]
        rko = rng.randint(0, 1)
        ra = oracle.jerasure_matrix_decode(k, m, M, rko, pat + [-1], A[:k], A[k:], B)
        rb = ecg.jerasure_matrix_decode(k, m, M, rko, pat + [-1], Bb[:k], Bb[k:], B)
        assert ra == rb and same(A, Bb), (k, m, M, pat, rko)


def test_matrix_dotprod(ecg, oracle, torch_cuda):
    """jerasure_matrix_dotprod (row a2): data sources or src_ids mixing data and coding blocks, any
    destination, coefficient 0/1/other; an all-zero row leaves the destination untouched."""
    rng = random.Random(11)
    for trial in range(40):
        k, m, B = rng.randint(1, 12), rng.randint(1, 5), rng.choice([1, 17, 1024, 4099])
        row = [rng.choice([0, 1, rng.randrange(256)]) for _ in range(k)]
        if trial % 7 == 0:
            row = [0] * k
        src = None if trial % 2 else [rng.randrange(k + m) for _ in range(k)]
        dest = rng.randrange(k + m)
        eff = [(src[i] if src else i) for i in range(k) if row[i]]
        if dest in eff:  # aliasing is refused (ECG_EINVAL), never computed
            data = [rnd(B, j) for j in range(k)]
            coding = [rnd(B, 99 + j) for j in range(m)]
            with pytest.raises(ecg.EcgError):
                ecg.jerasure_matrix_dotprod(k, row, src, dest, data, coding, B)
            continue
        data = [rnd(B, trial * 31 + j) for j in range(k)]
        coding = [rnd(B, 500 + trial * 31 + j) for j in range(m)]
        a = [x.copy() for x in data], [x.copy() for x in coding]
        b = [x.copy() for x in data], [x.copy() for x in coding]
        oracle.jerasure_matrix_dotprod(k, row, src, dest, a[0], a[1], B)
        ecg.jerasure_matrix_dotprod(k, row, src, dest, b[0], b[1], B)
        assert same(a[0] + a[1], b[0] + b[1]), (trial, k, row, src, dest)


def test_galois_region_xor(ecg, oracle, torch_cuda):
    for n in (1, 17, 4096, 4097, 100003):  # <= 4096: host coefficient rows; above: the GPU
        s, d = rnd(n, 1), rnd(n, 2)
        d2 = d.copy()
        oracle.galois_region_xor(s, d, n)
        ecg.galois_region_xor(s, d2, n)
        assert np.array_equal(d, d2)


# ------------------------------------------------------------------ ErasureCode facade vs oracle classes

GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def test_facade_encode_matches_golden(ecg, torch_cuda):
    B = GOLDEN["block_size"]
    for c in GOLDEN["codes"]:
        ec = ecg.ec_factory(c["type"], ecg.CodingParameters(**c["params"]))
        data = [np.frombuffer(bytes.fromhex(h), np.uint8).copy() for h in c["data_hex"]]
        coding = [np.zeros(B, np.uint8) for _ in range(ec.m)]
        assert ec.encode(data, coding, B) == 0
        assert [x.tobytes().hex() for x in coding] == c["coding_hex"], c["name"]


CODES = [(c["name"], c["type"], c["params"]) for c in GOLDEN["codes"]]


def _pair(t, params, local=False):
    from oracle import ec_ref as E
    import ecg as P
    cp = dict(params, local_or_column=local)
    o = E.ec_factory(t, E.CodingParameters(**cp))
    p = P.ec_factory(t, P.CodingParameters(**cp))
    o.local_or_column = local
    p.init_coding_parameters(P.CodingParameters(**cp)) if local else None
    if local and hasattr(o, "e_row_code"):  # HPC init also resets ERS parts
        o.init_coding_parameters(E.CodingParameters(**cp))
    return o, p


@pytest.mark.parametrize("name,t,params", CODES)
def test_facade_decode_vs_oracle(ecg, oracle, torch_cuda, name, t, params):
    rng = random.Random(name)
    B = 4096 + 5
    o, p = _pair(t, params)
    from oracle import ec_ref as E
    data = E.blocks(o.k, B, 77)
    coding = E.zeros(o.m, B)
    o.encode(data, coding, B)
    stripe = data + coding
    n = o.k + o.m
    for _ in range(12):
        pat = rng.sample(range(n), rng.randint(1, min(4, o.m)))
        A = [x.copy() for x in stripe]
        Bb = [x.copy() for x in stripe]
        for i in pat:
            A[i][:] = 0
            Bb[i][:] = 0
        ra = o.decode(A[:o.k], A[o.k:], B, pat + [-1], len(pat))  # -1-terminated (LRCs: the global path)
        rb = p.decode(Bb[:o.k], Bb[o.k:], B, pat + [-1], len(pat))
        assert (ra == 0) == (rb == 0), (pat, ra, rb)
        assert same(A, Bb), pat
    if t in (2, 3, 4, 5, 6):
        _lrc_local_decodes(E, t, params, stripe, B, rng)


def _lrc_local_decodes(E, t, params, stripe, B, rng):
    """The LRC local path of ErasureCode::decode (lrc.cpp:32-42,58-72), as main_repair calls it without partial
    decoding (handle_repair.cpp:377-384): local_or_column set, the group's blocks in group space (data_ptrs:
    the group_size members, coding_ptrs: its local parity), erasures = [index in the group, group_id] with
    failed_num = 1 -- group_id rides in erasures[failed_num] (handle_repair.cpp:380-381) and comes back as -1.
    Every position of every group (the local parity included), plus random positions with garbage in the
    lost block; status and every byte against the oracle.  (The Cauchy LRCs' group rows are not all ones, so
    some of their lost data blocks come back wrong in both -- Appendix B.1, test_cauchy_local_decode_quirk.)"""
    o, p = _pair(t, params, local=True)
    k, g, l = o.k, o.g, o.l
    for gid in range(l):
        gs, mn = o.get_group_size(gid)
        members = (list(range(mn, mn + gs - g)) + list(range(k, k + g))) if t == 5 else list(range(mn, mn + gs))
        group = [stripe[b] for b in members] + [stripe[k + g + gid]]
        for lost in list(range(gs + 1)) + [rng.randrange(gs + 1) for _ in range(2)]:
            A = [x.copy() for x in group]
            Bq = [x.copy() for x in group]
            A[lost][:] = 0xD1
            Bq[lost][:] = 0xD1
            ea, eb = [lost, gid], [lost, gid]
            ra = o.decode(A[:gs], A[gs:], B, ea, 1)
            rb = p.decode(Bq[:gs], Bq[gs:], B, eb, 1)
            assert (ra == 0) == (rb == 0), (t, gid, lost, ra, rb)
            assert eb == [lost, -1], eb  # lrc.cpp:36: the group id slot is overwritten with -1
            assert same(A, Bq), (t, gid, lost)
            if t not in (5, 6):  # all-ones group rows: the local decode rebuilds the lost block
                assert np.array_equal(Bq[lost], group[lost]), (t, gid, lost)


@pytest.mark.parametrize("name,t,params", CODES)
def test_facade_partials_vs_oracle(ecg, oracle, torch_cuda, name, t, params):
    from oracle import ec_ref as E
    rng = random.Random(name + "p")
    B = 1000
    for local in (False, True):
        o, p = _pair(t, params, local)
        if local and t in (0, 1):
            continue
        data = E.blocks(o.k, B, 3)
        coding = E.zeros(o.m, B)
        o.encode(data, coding, B)
        stripe = data + coding
        k, m = o.k, o.m
        for _ in range(6):
            if t >= 7:  # product codes: one row (or column) of the grid
                if not local:
                    r = rng.randrange(o.k2)
                    members = [o.rowcol2bid(r, c) for c in range(o.k1 + o.m1)]
                    nd = o.k1
                else:
                    c = rng.randrange(o.k1)
                    members = [o.rowcol2bid(r, c) for r in range(o.k2 + o.m2)]
                    nd = o.k2
                d_all, par = members[:nd], members[nd:]
            elif local:
                gid = rng.randrange(o.l)
                gs, mn = o.get_group_size(gid)
                if name.startswith("OptCauchy"):
                    d_all = list(range(mn, mn + gs - o.g)) + list(range(k, k + o.g))
                else:
                    d_all = list(range(mn, mn + gs))
                par = [k + o.g + gid]
            else:
                d_all, par = list(range(k)), list(range(k, k + (o.g if hasattr(o, "g") else m)))
            cut = rng.randint(1, len(d_all) - 1) if len(d_all) > 1 else 1
            sub = rng.sample(d_all, cut)
            outs_a, outs_b = E.zeros(len(par), B), E.zeros(len(par), B)
            o.encode_partial_blocks_for_encoding([stripe[i] for i in sub], outs_a, B, sub, par)
            p.encode_partial_blocks_for_encoding([stripe[i] for i in sub], outs_b, B, sub, par)
            assert same(outs_a, outs_b), ("enc", local, sub, par)
            # partial decoding: lose one member, survivors = the rest (exactly k' of them)
            group = d_all + par
            lost = rng.choice(group)
            surv = [i for i in group if i != lost][:len(d_all)]
            lsub = rng.sample(surv, rng.randint(1, len(surv)))
            da, db = E.zeros(1, B), E.zeros(1, B)
            o.encode_partial_blocks_for_decoding([stripe[i] for i in lsub], da, B, lsub, surv, [lost])
            p.encode_partial_blocks_for_decoding([stripe[i] for i in lsub], db, B, lsub, surv, [lost])
            assert same(da, db), ("dec", local, lsub, surv, lost)


def test_config3_full_block_repairs(ecg, torch_cuda):
    """BASELINE config 3 at its block size: Azure-LRC(12,2,2), 1 MiB blocks, single-block repair with
    partial decoding for every local block (data and local parities), as the proxies issue it per stripe
    (helper partial, main partial, perform_addition; handle_repair.cpp:249,371-376) -- once with the
    partials in HBM and once composed away (batch_scratch).  Every repaired block must equal the lost one."""
    torch = torch_cuda
    S, B = 14, 1 << 20
    ec, st, plan = _azure_repair_state(ecg, torch, S, B, 0xC3)
    idx = torch.arange(S, device="cuda")
    want = st[idx, torch.tensor([p[0] for p in plan], device="cuda")]
    for scratch in (False, True):
        partials = torch.full((S, 2, B), 0x77, dtype=torch.uint8, device="cuda")
        out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
        with ecg.batch() as scope:
            if scratch:
                scope.scratch(partials)
            _repair_sequence(ec, st, plan, partials, out, B)
        torch.cuda.synchronize()
        assert torch.equal(out, want), scratch
        assert bool((partials == 0x77).all()) == scratch


def test_config4_full_block_merge(ecg, oracle, torch_cuda):
    """BASELINE config 4 at its block size: two PC(4,1,4,1) stripes with 4 MiB blocks merged (x = 2,
    horizontal) into PC(8,1,4,1).  Each data row's new row parity is two partial encodings of the
    merged code (one per old stripe's half of the row, erasure_code.cpp:97-111 with the new stripe's block
    ids, merge.cpp:82) plus perform_addition at the parity's proxy (handle_merge.cpp:159,319), on HBM
    blocks in one batch scope with the partials as scratch.  Compared with the oracle's encoding of the
    merged stripe."""
    from oracle import ec_ref as E
    torch = torch_cuda
    B = 4 << 20
    old = E.ec_factory(7, E.CodingParameters(k1=4, m1=1, k2=4, m2=1))
    new_o = E.ec_factory(7, E.CodingParameters(k1=8, m1=1, k2=4, m2=1))
    new_p = ecg.ec_factory(ecg.ECTYPE.PC, ecg.CodingParameters(k1=8, m1=1, k2=4, m2=1))
    halves = [E.blocks(old.k, B, 40 + h) for h in range(2)]  # data of the two old stripes, row-major 4 x 4
    # merged data in the new code's block-id order
    data_new = [None] * new_o.k
    for r in range(4):
        for c in range(8):
            data_new[new_o.rowcol2bid(r, c)] = halves[c // 4][old.rowcol2bid(r, c % 4)]
    coding = E.zeros(new_o.m, B)
    new_o.encode(data_new, coding, B)
    stripe_new = data_new + coding
    d_half = [torch.from_numpy(np.stack(h)).cuda() for h in halves]
    partials = torch.full((4, 2, B), 0x5D, dtype=torch.uint8, device="cuda")
    out = torch.zeros((4, B), dtype=torch.uint8, device="cuda")
    with ecg.batch() as scope:
        scope.scratch(partials)
        for r in range(4):
            par = [new_o.rowcol2bid(r, 8)]
            for h in range(2):
                ids = [new_o.rowcol2bid(r, 4 * h + c) for c in range(4)]
                blocks = [d_half[h][old.rowcol2bid(r, c)] for c in range(4)]
                assert new_p.encode_partial_blocks_for_encoding(blocks, [partials[r, h]], B, ids, par) == 0
            assert new_p.perform_addition([partials[r, 0], partials[r, 1]], [out[r]], B, 2, 1) == 0
    torch.cuda.synchronize()
    assert bool((partials == 0x5D).all())
    for r in range(4):
        assert np.array_equal(out[r].cpu().numpy(), stripe_new[new_o.rowcol2bid(r, 8)]), r


def test_partial_plan_cache_tells_objects_apart(ecg, oracle, torch_cuda):
    """The per-thread plan cache of the partial calls is keyed by each object's state (class, parameters,
    sub-codes): objects of one class that differ only in a parameter the matrices depend on -- ERS
    seri_num, HPC isvertical, RS vs ERS with the same k and m -- alternate on one thread with identical
    index lists, and every result must still be its own object's (oracle)."""
    from oracle import ec_ref as E
    B = 512
    pairs = [(1, dict(k=4, m=2, x=2, seri_num=0), dict(k=4, m=2, x=2, seri_num=1)),
             (1, dict(k=4, m=2, x=2, seri_num=1), dict(k=4, m=2, x=3, seri_num=1)),
             (0, dict(k=4, m=2), None),  # RS vs ERS(4, 2, x=2, seri_num=1) below
             (8, dict(k1=2, m1=2, k2=2, m2=1, x=2, seri_num=1), "vertical")]
    for t, pa, pb in pairs:
        if pb is None:
            objs = [(0, pa, None), (1, dict(k=4, m=2, x=2, seri_num=1), None)]
        elif pb == "vertical":
            objs = [(t, pa, True), (t, pa, False)]
        else:
            objs = [(t, pa, None), (t, pb, None)]
        built = []
        for tt, pp, vert in objs:
            o = E.ec_factory(tt, E.CodingParameters(**pp))
            p = ecg.ec_factory(tt, ecg.CodingParameters(**pp))
            p.init_coding_parameters(ecg.CodingParameters(**pp))
            o.init_coding_parameters(E.CodingParameters(**pp))
            if vert is not None:
                o.isvertical = vert
                p.set_isvertical(vert)
            built.append((o, p))
        o0 = built[0][0]
        k, m = o0.k, o0.m
        if t >= 7:  # product code: one row of the grid
            members = [o0.rowcol2bid(0, c) for c in range(o0.k1 + o0.m1)]
            d_all, par = members[:o0.k1], members[o0.k1:]
        else:
            d_all, par = list(range(k)), list(range(k, k + m))
        sub = d_all[1:]
        lost = [d_all[0]]
        surv = (d_all[1:] + par)[:len(d_all)]
        for rep in range(3):  # alternate: a stale cache entry would hand one object the other's plan
            for o, p in built:
                stripe = E.blocks(k, B, 11) + E.zeros(m, B)
                o.encode(stripe[:k], stripe[k:], B)
                a, b = E.zeros(len(par), B), E.zeros(len(par), B)
                o.encode_partial_blocks_for_encoding([stripe[i] for i in sub], a, B, sub, par)
                p.encode_partial_blocks_for_encoding([stripe[i] for i in sub], b, B, sub, par)
                assert same(a, b), (t, rep, "enc")
                da, db = E.zeros(1, B), E.zeros(1, B)
                o.encode_partial_blocks_for_decoding([stripe[i] for i in surv[:2]], da, B, surv[:2], surv, lost)
                p.encode_partial_blocks_for_decoding([stripe[i] for i in surv[:2]], db, B, surv[:2], surv, lost)
                assert same(da, db), (t, rep, "dec")


@pytest.mark.parametrize("t,params,local", [(0, dict(k=10, m=4), False), (0, dict(k=6, m=4), False),
                                             (2, dict(k=12, l=2, g=2), True), (2, dict(k=12, l=2, g=2), False)])
def test_main_repair_with_addition(ecg, oracle, torch_cuda, t, params, local):
    """encode_partial_blocks_for_decoding_with_addition == the main proxy's own partial followed by
    perform_addition over [helper partials..., own partials] (handle_repair.cpp:371-376), and == the lost
    blocks; also with no local blocks (pure addition) and no helper partials (own partial only)."""
    from oracle import ec_ref as E
    rng = random.Random(t * 10 + params["k"] + local)
    B = 4096 + 3
    o, p = _pair(t, params, local)
    data = E.blocks(o.k, B, 5)
    coding = E.zeros(o.m, B)
    o.encode(data, coding, B)
    stripe = data + coding
    for trial in range(8):
        if local:
            gid = rng.randrange(o.l)
            gs, mn = o.get_group_size(gid)
            group = list(range(mn, mn + gs)) + [o.k + o.g + gid]
            f = 1
        else:
            group = list(range(o.k)) + list(range(o.k, o.k + (o.g if hasattr(o, "g") else o.m)))
            f = rng.randint(1, min(3, len(group) - o.k))
        lost = rng.sample(group, f)
        need = len(group) - 1 if local else o.k  # encode_partial_blocks_for_decoding takes exactly k' survivors
        surv = [i for i in group if i not in lost][:need]
        parts = [[], [], []]
        for i in surv:
            parts[rng.randrange(3)].append(i)
        if trial == 0:
            parts = [surv[:len(surv) // 2], surv[len(surv) // 2:], []]  # main holds no block
        if trial == 1:
            parts = [[], [], surv]                                        # no helper partials
        helper_partials = []
        for h in parts[:2]:
            if h:
                out = E.zeros(f, B)
                o.encode_partial_blocks_for_decoding([stripe[i] for i in h], out, B, h, surv, lost)
                helper_partials += out
        mine = parts[2]
        expect = E.zeros(f, B)
        if mine:
            own = E.zeros(f, B)
            o.encode_partial_blocks_for_decoding([stripe[i] for i in mine], own, B, mine, surv, lost)
        else:
            own = []
        allp = helper_partials + own
        if len(allp) == f:
            expect = allp
        else:
            o.perform_addition(allp, expect, B, len(allp), f)
        got = [np.full(B, 0x77, np.uint8) for _ in range(f)]
        assert p.encode_partial_blocks_for_decoding_with_addition(
            [stripe[i] for i in mine], helper_partials, got, B, mine, surv, lost) == 0
        assert same(got, expect), (trial, parts, lost)
        assert same(got, [stripe[i] for i in lost]), (trial, parts, lost)
    # device tier, same call on HBM buffers
    torch = torch_cuda
    mine, hp_host = surv[:2], E.zeros(f, B)
    rest = surv[2:]
    o.encode_partial_blocks_for_decoding([stripe[i] for i in rest], hp_host, B, rest, surv, lost)
    d_loc = [torch.from_numpy(stripe[i]).cuda() for i in mine]
    d_hp = [torch.from_numpy(x).cuda() for x in hp_host]
    d_out = [torch.zeros(B, dtype=torch.uint8, device="cuda") for _ in range(f)]
    assert p.encode_partial_blocks_for_decoding_with_addition(d_loc, d_hp, d_out, B, mine, surv, lost) == 0
    torch.cuda.synchronize()
    assert same([x.cpu().numpy() for x in d_out], [stripe[i] for i in lost])


@pytest.mark.parametrize("t,params", [(0, dict(k=10, m=4)), (1, dict(k=4, m=2, x=3, seri_num=1)),
                                      (2, dict(k=12, l=2, g=2))])
def test_merge_recal_with_addition(ecg, oracle, torch_cuda, t, params):
    """encode_partial_blocks_for_encoding_with_addition == the parity proxy's own partial encoding
    followed by perform_addition over [helper partials..., own partials] (handle_merge.cpp:159,319), and
    == the full parities when the parts cover all data."""
    from oracle import ec_ref as E
    rng = random.Random(t * 7 + params["k"])
    B = 2048 + 9
    o, p = _pair(t, params)
    data = E.blocks(o.k, B, 9)
    coding = E.zeros(o.m, B)
    o.encode(data, coding, B)
    stripe = data + coding
    npar = o.g if hasattr(o, "g") else o.m
    for trial in range(6):
        par = sorted(rng.sample(range(o.k, o.k + npar), rng.randint(1, npar)))
        parts = [[], [], []]
        for i in range(o.k):
            parts[rng.randrange(3)].append(i)
        if trial == 0:
            parts = [list(range(o.k)), [], []]
        helper_partials = []
        for h in parts[:2]:
            if h:
                out = E.zeros(len(par), B)
                o.encode_partial_blocks_for_encoding([stripe[i] for i in h], out, B, h, par)
                helper_partials += out
        mine = parts[2]
        own = []
        if mine:
            own = E.zeros(len(par), B)
            o.encode_partial_blocks_for_encoding([stripe[i] for i in mine], own, B, mine, par)
        allp = helper_partials + own
        expect = E.zeros(len(par), B)
        o.perform_addition(allp, expect, B, len(allp), len(par))
        got = [np.full(B, 0x11, np.uint8) for _ in par]
        assert p.encode_partial_blocks_for_encoding_with_addition(
            [stripe[i] for i in mine], helper_partials, got, B, mine, par) == 0
        assert same(got, expect), (trial, parts, par)
        assert same(got, [stripe[i] for i in par]), (trial, parts, par)


def test_perform_addition(ecg, oracle, torch_cuda):
    from oracle import ec_ref as E
    o = E.RSCode(4, 2)
    p = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=4, m=2))
    for n, par, B in [(2, 1, 1 << 20), (6, 2, 1001), (12, 4, 64), (9, 3, 16)]:
        parts = [rnd(B, 10 * i + n) for i in range(n)]
        a, b = E.zeros(par, B), E.zeros(par, B)
        o.perform_addition(parts, a, B, n, par)
        assert p.perform_addition(parts, b, B, n, par) == 0
        assert same(a, b)


def test_lrc_local_decode_side_channel(ecg, oracle, torch_cuda):
    """LRC local decode: group_id rides in erasures[failed_num] and is overwritten with -1 (lrc.cpp:35-38)."""
    from oracle import ec_ref as E
    B = 4096
    o, p = _pair(2, dict(k=12, l=2, g=2), local=True)
    data = E.blocks(12, B, 1)
    coding = E.zeros(4, B)
    o.encode(data, coding, B)
    group = data[6:12] + [coding[3]]  # group 1: blocks 6..11, local parity 15
    for lost in range(6):
        A = [x.copy() for x in group]
        A[lost][:] = 0
        er = [lost, 1]
        assert p.decode(A[:6], A[6:], B, er, 1) == 0
        assert er == [lost, -1]
        assert np.array_equal(A[lost], group[lost])


@pytest.mark.parametrize("t", [5, 6])  # OPTIMAL_CAUCHY_LRC, UNIFORM_CAUCHY_LRC
def test_cauchy_local_decode_quirk(ecg, oracle, torch_cuda, t):
    """decode_local hands failed_num to jerasure_matrix_decode as row_k_ones (lrc.cpp:58-71).  The Cauchy
    LRCs' group rows are not all ones, so Jerasure's "last drive" XOR shortcut rebuilds a lost data block
    wrongly — the engine must reproduce the reference's (wrong) bytes exactly, not silently fix them."""
    from oracle import ec_ref as E
    B = 1024
    o, p = _pair(t, dict(k=8, l=2, g=2), local=True)
    gs, _ = o.get_group_size(0)
    row = o.make_group_matrix(0, gs)
    assert any(c != 1 for c in row)  # the premise of the quirk
    group = E.blocks(gs, B, 3)
    local = E.zeros(1, B)
    oracle.jerasure_matrix_encode(gs, 1, row, group, local, B)
    wrong = 0
    for lost in range(gs):
        A = [x.copy() for x in group] + [local[0].copy()]
        Bq = [x.copy() for x in A]
        A[lost][:] = 0
        Bq[lost][:] = 0
        o.decode(A[:gs], A[gs:], B, [lost, 0], 1)
        assert p.decode(Bq[:gs], Bq[gs:], B, [lost, 0], 1) == 0
        assert np.array_equal(A[lost], Bq[lost]), lost  # bit-exact with the reference restatement
        wrong += not np.array_equal(Bq[lost], group[lost])
    assert wrong > 0  # and the quirk is real: some lost blocks come back wrong, as in the reference


# ------------------------------------------------------------------ device tier + batches

@pytest.mark.parametrize("lat_dword", [None, 0])
def test_device_tier_single_call_latency_kernel(ecg, oracle, torch_cuda, lat_dword):
    """Single device-tier calls with blocks up to ECG_OPT_LAT_DWORD_BYTES run the latency kernel (4 bytes
    per lane, every input-count bucket, padded inputs masked); above it, or with the option at 0, the
    bulk kernel.  Both against the oracle, back to back on one stream, then one synchronize."""
    torch = torch_cuda
    saved = ecg.get_option(ecg.ECG_OPT_LAT_DWORD_BYTES)
    if lat_dword is not None:
        ecg.set_option(ecg.ECG_OPT_LAT_DWORD_BYTES, lat_dword)
    try:
        rng = random.Random(5)
        cases = []
        for B in (1024, 65536, 65552, 262144, 1 << 20, (1 << 20) + 16):
            for k in (1, 3, 5, 6, 7, 10, 12, 13, 16, 17):
                m = rng.randint(1, 9)
                M = ([rng.randrange(2) for _ in range(k * m)] if k % 2 else
                     [rng.randrange(256) for _ in range(k * m)])
                host = [rnd(B, 300 * k + j + B) for j in range(k)]
                dev_data = [torch.from_numpy(h).cuda() for h in host]
                dev_cod = [torch.zeros(B, dtype=torch.uint8, device="cuda") for _ in range(m)]
                ecg.dev_matrix_encode(k, m, M, dev_data, dev_cod, B)
                cases.append((B, k, m, M, host, dev_cod))
        # many outputs: several row tiles per call, up to the 32 inline output pointers (each tile reads its
        # own tables and output pointers)
        for B, k, m in ((65536, 4, 17), (65536, 16, 32), (4096, 10, 24), (1 << 20, 12, 32)):
            for binary in (False, True):
                M = [rng.randrange(2) if binary else rng.randrange(256) for _ in range(k * m)]
                host = [rnd(B, 77 * k + j + m) for j in range(k)]
                dev_data = [torch.from_numpy(h).cuda() for h in host]
                dev_cod = [torch.zeros(B, dtype=torch.uint8, device="cuda") for _ in range(m)]
                ecg.dev_matrix_encode(k, m, M, dev_data, dev_cod, B)
                cases.append((B, k, m, M, host, dev_cod))
        torch.cuda.synchronize()
        for B, k, m, M, host, dev_cod in cases:
            ref = [np.zeros(B, np.uint8) for _ in range(m)]
            oracle.jerasure_matrix_encode(k, m, M, host, ref, B)
            assert same([c.cpu().numpy() for c in dev_cod], ref), (B, k, m)
    finally:
        ecg.set_option(ecg.ECG_OPT_LAT_DWORD_BYTES, saved)


def test_device_tier_aligned_and_unaligned(ecg, oracle, torch_cuda):
    torch = torch_cuda
    k, m = 10, 4
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    for B, off in [(65536, 0), (4099, 0), (4096, 1), (777, 3)]:
        host = [rnd(B, j + B) for j in range(k)]
        dev_data = [torch.from_numpy(np.concatenate([np.zeros(off, np.uint8), h])).cuda()[off:] for h in host]
        dev_cod = [torch.zeros(B + off, dtype=torch.uint8, device="cuda")[off:] for _ in range(m)]
        ecg.dev_matrix_encode(k, m, M, dev_data, dev_cod, B)
        torch.cuda.synchronize()
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, host, ref, B)
        assert same([c.cpu().numpy() for c in dev_cod], ref), (B, off)
        # decode on device, in place
        for pat in ([3], [0, 11], [10, 12, 13, 1]):
            dd = [d.clone() for d in dev_data] + [c.clone() for c in dev_cod]
            for i in pat:
                dd[i].fill_(0)
            assert ecg.dev_matrix_decode(k, m, M, 1, pat + [-1], dd[:k], dd[k:], B) == 0
            torch.cuda.synchronize()
            assert same([x.cpu().numpy() for x in dd], host + ref), pat


def test_facade_device_tier(ecg, oracle, torch_cuda):
    torch = torch_cuda
    from oracle import ec_ref as E
    B = 8192
    for name, t, params in CODES:
        o, p = _pair(t, params)
        data = E.blocks(o.k, B, 5)
        coding = E.zeros(o.m, B)
        o.encode(data, coding, B)
        dd = [torch.from_numpy(x).cuda() for x in data]
        dc = [torch.zeros(B, dtype=torch.uint8, device="cuda") for _ in range(o.m)]
        assert p.encode(dd, dc, B) == 0
        torch.cuda.synchronize()
        assert same([c.cpu().numpy() for c in dc], coding), name


def test_fill_random_matches_oracle(ecg, oracle, torch_cuda):
    torch = torch_cuda
    for n, off in [(1, 0), (13, 5), (1 << 20, 123456)]:
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        ecg.fill_random(t, 0xEC0DE, off)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), oracle.splitmix_bytes(0xEC0DE, off, n))


@pytest.mark.parametrize("k,m,B,S", [(10, 4, 1 << 20, 6), (13, 5, 65536 + 40, 5), (9, 7, 65536 + 40, 3),
                                     (3, 9, 4096 + 8, 4), (11, 12, 4096 + 8, 3)])
def test_encode_batch_vs_oracle(ecg, oracle, torch_cuda, k, m, B, S):
    """Strided batched encodes: the headline shape, and GENERAL tiles of 5+ outputs (two inputs per load batch)
    with odd input counts -- the single-input tail after the pairs -- and two row tiles (m = 9, 12), with byte
    tails (B % 16 != 0 goes to the byte kernel)."""
    torch = torch_cuda
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    d_in = torch.empty((S, k, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(d_in, 7)
    d_out = torch.empty((S, m, B), dtype=torch.uint8, device="cuda")
    ecg.encode_batch(k, m, M, d_in, d_out)
    torch.cuda.synchronize()
    hin, hout = d_in.cpu().numpy(), d_out.cpu().numpy()
    for s in range(S):
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode_simd(k, m, M, [hin[s, j] for j in range(k)], ref, B)
        assert same([hout[s, i] for i in range(m)], ref), s


def test_decode_batch_rotating_patterns(ecg, oracle, torch_cuda):
    torch = torch_cuda
    k, m, B, S = 10, 4, 65536 + 16, 28
    n = k + m
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes[:, :k], 1)  # non-contiguous view fill is not allowed -> fill whole then encode
    ecg.fill_random(stripes, 1)
    ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])
    patterns = [[e] for e in range(n)]
    pos = torch.arange(S, device="cuda", dtype=torch.int32) % n
    out = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    # the erased block of every stripe is saved, then POISONED: a decode that read it (or copied it) fails
    sidx = torch.arange(S, device="cuda")
    saved = stripes[sidx, sidx % n].clone()
    stripes[sidx, sidx % n] = 0xA5
    ecg.decode_batch(k, m, M, 1, patterns, stripes, out=out, pattern_of_stripe=pos)
    torch.cuda.synchronize()
    assert torch.equal(out[:, 0], saved)
    # byte for byte against the oracle's decode of the poisoned stripe (erased block = output)
    for s in (0, 5, 13, S - 1):
        h = [x.copy() for x in stripes[s].cpu().numpy()]
        assert oracle.jerasure_matrix_decode(k, m, M, 1, [s % n, -1], h[:k], h[k:], B) == 0
        assert np.array_equal(out[s, 0].cpu().numpy(), h[s % n]), s
    # the check can fail: a plan that READS the poisoned block gives other bytes.  Rebuilding e + 1 reads
    # the first k surviving blocks, which include e whenever e is a data block (e < k)
    shifted = [[(e + 1) % n] for e in range(n)]
    bad = torch.empty_like(out)
    ecg.decode_batch(k, m, M, 1, shifted, stripes, out=bad, pattern_of_stripe=pos)
    torch.cuda.synchronize()
    nxt = stripes[sidx, (sidx + 1) % n]
    for s in range(S):
        assert torch.equal(bad[s, 0], nxt[s]) == (s % n >= k), s
    stripes[sidx, sidx % n] = saved
    # in place, pairs of erasures, stripes padded (block stride > B)
    pad = torch.zeros((4, n, B + 48), dtype=torch.uint8, device="cuda")
    view = pad[:, :, :B]
    view.copy_(stripes[:4])
    orig = view.clone()
    view[:, 2].zero_()
    view[:, 12].zero_()
    ecg.decode_batch(k, m, M, 1, [[2, 12]], view)
    torch.cuda.synchronize()
    assert torch.equal(view, orig)


def test_matrix_apply_and_addition_batch(ecg, oracle, torch_cuda):
    torch = torch_cuda
    B, S = 4096, 16
    d_in = torch.empty((S, 6, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(d_in, 9)
    coef = [[1, 7, 0, 255], [0, 0, 1, 1]]
    out = torch.zeros((S, 3, B), dtype=torch.uint8, device="cuda")
    ecg.matrix_apply_batch(coef, [5, 1, 2, 0], [2, 0], d_in, out)
    add = torch.zeros((S, 2, B), dtype=torch.uint8, device="cuda")
    ecg.perform_addition_batch(6, 2, d_in, add)
    torch.cuda.synchronize()
    hin, hout, hadd = d_in.cpu().numpy(), out.cpu().numpy(), add.cpu().numpy()
    for s in range(S):
        src = [hin[s, i] for i in (5, 1, 2, 0)]
        ref = [np.zeros(B, np.uint8) for _ in range(2)]
        oracle.jerasure_matrix_encode(4, 2, [c for r in coef for c in r], src, ref, B)
        assert np.array_equal(hout[s, 2], ref[0]) and np.array_equal(hout[s, 0], ref[1])
        assert not hout[s, 1].any()
        for i in range(2):
            assert np.array_equal(hadd[s, i], hin[s, i] ^ hin[s, i + 2] ^ hin[s, i + 4])


def test_threads_concurrent_host_calls(ecg, oracle, torch_cuda):
    """The proxy runs EC calls on detached threads (proxy.cpp:416-419): concurrent host-tier calls."""
    k, m, B = 6, 4, 1 << 16
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    errors = []

    def worker(t):
        try:
            for it in range(5):
                data = [rnd(B, 1000 * t + 10 * it + j) for j in range(k)]
                a = [np.zeros(B, np.uint8) for _ in range(m)]
                b = [np.zeros(B, np.uint8) for _ in range(m)]
                oracle.jerasure_matrix_encode(k, m, M, data, a, B)
                ecg.jerasure_matrix_encode(k, m, M, data, b, B)
                if not same(a, b):
                    errors.append((t, it))
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    [x.start() for x in th]
    [x.join() for x in th]
    assert not errors


def test_full_size_rs10_4_round_trip(ecg, oracle, torch_cuda):
    """BASELINE config 2 at full size: RS(10,4), 1 MiB blocks, 4096 stripes (56 GiB in HBM).
    encode -> rotate one erasure per stripe (s mod 14) -> decode -> equals the original block; three
    sampled stripes also checked byte-for-byte against the oracle."""
    torch = torch_cuda
    k, m, B, S = 10, 4, 1 << 20, 4096
    n = k + m
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 0xEC0DE)
    ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    out = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    sidx = torch.arange(S, device="cuda")
    idx = sidx % n
    samples = (0, 1234, S - 1)
    for s in samples:  # parities of sampled stripes against the oracle, before any block is poisoned
        h = stripes[s].cpu().numpy()
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode_simd(k, m, M, [h[j] for j in range(k)], ref, B)
        assert same([h[k + i] for i in range(m)], ref), s
    # the erased block (s mod 14) is saved, then poisoned in place: the decode must not read it
    expect = stripes[sidx, idx].clone()
    stripes[sidx, idx] = 0x5A
    ecg.decode_batch(k, m, M, 1, [[e] for e in range(n)], stripes, out=out, pattern_of_stripe=pos)
    torch.cuda.synchronize()
    assert torch.equal(out[:, 0], expect)
    for s in samples:  # the oracle decodes the same poisoned stripe to the same bytes
        h = [x.copy() for x in stripes[s].cpu().numpy()]
        assert oracle.jerasure_matrix_decode(k, m, M, 1, [s % n, -1], h[:k], h[k:], B) == 0
        assert np.array_equal(out[s, 0].cpu().numpy(), h[s % n]), s
    del stripes, out, expect
    torch.cuda.empty_cache()


def test_config5_waves_sharded(ecg, oracle, torch_cuda):
    """BASELINE config 5 (RS(10,4), 4 MiB blocks, a stripe batch sharded over GPUs and encoded in
    HBM-resident waves) through bench.py's own encode_waves at a small size: 67 stripes, waves of 32.
    Sampled stripes (first / last of a wave, both shard edges) are compared byte for byte with the oracle
    on host-generated data, and the per-rank parity checksums of a 2-way and a 3-way split, combined,
    equal the unsplit checksum (the SCALE run's bit-exact verdict)."""
    torch = torch_cuda
    import ecg_dist as D
    from bench import encode_waves
    k, m, B, total, W = 10, 4, 4 << 20, 67, 32
    n = k + m
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    sample = {0, 31, 32, 33, 34, 44, 45, 66}
    checked = set()

    def check(s0, buf):
        for s in range(s0, s0 + buf.shape[0]):
            if s not in sample or s in checked:
                continue
            h = buf[s - s0].cpu().numpy()
            data = [oracle.splitmix_bytes(0xEC0DE, (s * n + j) * B // 8, B) for j in range(k)]
            assert same([h[j] for j in range(k)], data), f"stripe {s}: device data != host splitmix"
            ref = [np.zeros(B, np.uint8) for _ in range(m)]
            oracle.jerasure_matrix_encode_simd(k, m, M, data, ref, B)
            assert same([h[k + i] for i in range(m)], ref), f"stripe {s}: parity mismatch"
            checked.add(s)

    _, whole = encode_waves(k, m, M, B, 0, total, W, on_wave=check)
    assert checked == sample
    for world in (2, 3):
        parts = []
        for rank in range(world):
            first, last = D.stripe_range(total, D.Rank(rank, world, rank))
            parts.append(encode_waves(k, m, M, B, first, last, W)[1])
        assert D.combine(parts) == whole, world
    torch.cuda.empty_cache()


def test_matrix_apply_multi_with_stripe_subset(ecg, oracle, torch_cuda):
    """Several programs per launch + launch over a subset of the batch (stripe_of indirection)."""
    torch = torch_cuda
    rng = random.Random(11)
    S, n, B = 24, 8, 4096 + 16
    d_in = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(d_in, 21)
    out = torch.zeros((S, 2, B), dtype=torch.uint8, device="cuda")
    progs = []
    for _ in range(5):
        src = rng.sample(range(n), 3)
        coef = [[rng.randrange(256) for _ in range(3)] for _ in range(2)]
        progs.append((coef, src, [1, 0]))
    subset = sorted(rng.sample(range(S), 11))
    which = [rng.randrange(5) for _ in subset]
    st = torch.tensor(subset, dtype=torch.int32, device="cuda")
    pp = torch.tensor(which, dtype=torch.int32, device="cuda")
    ecg.matrix_apply_batch_multi(progs, d_in, out, prog_of_stripe=pp, stripe_of=st)
    torch.cuda.synchronize()
    hin, hout = d_in.cpu().numpy(), out.cpu().numpy()
    for s in range(S):
        if s not in subset:
            assert not hout[s].any(), s
            continue
        coef, src, dst = progs[which[subset.index(s)]]
        ref = [np.zeros(B, np.uint8) for _ in range(2)]
        oracle.jerasure_matrix_encode(3, 2, [c for r in coef for c in r], [hin[s, j] for j in src], ref, B)
        assert np.array_equal(hout[s, 1], ref[0]) and np.array_equal(hout[s, 0], ref[1]), s


def _apply_ref(oracle, progs, which, hin, S, B, out_rows):
    """Host reference of matrix_apply_batch_multi: program which[s] of stripe s, all reads before writes."""
    ref = np.zeros((S, out_rows, B), np.uint8)
    for s in range(S):
        coef, src, dst = progs[which[s]]
        outs = [np.zeros(B, np.uint8) for _ in dst]
        oracle.jerasure_matrix_encode(len(src), len(dst), [c for r in coef for c in r], [hin[s, j] for j in src],
                                      outs, B)
        for p, d in enumerate(dst):
            ref[s, d] = outs[p]
    return ref


@pytest.mark.parametrize("split", [16, 0])
def test_row_split_of_separable_programs(ecg, oracle, torch_cuda, split):
    """ECG_OPT_ROW_SPLIT (engine.cpp row_split): programs whose output rows read disjoint input sets of one
    size run one launch stripe per (stripe, row).  Same bytes as the unsplit launch, for a BINARY 40 -> 5 PC
    merge shape, a GENERAL 16 -> 2 with two programs per launch over a stripe subset, tails and unaligned
    block sizes; and an in-place op whose outputs are inputs of other rows is never split (its rows must all
    read before any writes)."""
    torch = torch_cuda
    saved = ecg.get_option(ecg.ECG_OPT_ROW_SPLIT)
    rng = random.Random(5)
    try:
        ecg.set_option(ecg.ECG_OPT_ROW_SPLIT, split)
        # BINARY 40 -> 5, outputs in their own buffer
        S, n, B = 9, 50, 65536 + 48
        d_in = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(d_in, 31)
        src = rng.sample(range(n), 40)
        coef = [[1 if j // 8 == r else 0 for j in range(40)] for r in range(5)]
        progs = [(coef, src, [4, 0, 3, 1, 2])]
        out = torch.zeros((S, 5, B), dtype=torch.uint8, device="cuda")
        ecg.matrix_apply_batch_multi(progs, d_in, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), _apply_ref(oracle, progs, [0] * S, d_in.cpu().numpy(), S, B, 5))
        # GENERAL 16 -> 2, two programs (different row supports), stripe subset, B not a multiple of 16
        S, n, B = 20, 24, 4096 + 5
        d_in = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(d_in, 32)
        progs = []
        for _ in range(2):
            src = rng.sample(range(n), 16)
            cf = [[rng.randrange(1, 256) if (j < 8) == (r == 0) else 0 for j in range(16)] for r in range(2)]
            progs.append((cf, src, [1, 0]))
        subset = sorted(rng.sample(range(S), 13))
        which = [rng.randrange(2) for _ in subset]
        out = torch.zeros((S, 2, B), dtype=torch.uint8, device="cuda")
        ecg.matrix_apply_batch_multi(progs, d_in, out, prog_of_stripe=torch.tensor(which, dtype=torch.int32,
                                                                                    device="cuda"),
                                     stripe_of=torch.tensor(subset, dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        hin, hout = d_in.cpu().numpy(), out.cpu().numpy()
        wfull = [0] * S
        for s, w in zip(subset, which):
            wfull[s] = w
        ref = _apply_ref(oracle, progs, wfull, hin, S, B, 2)
        for s in range(S):
            assert np.array_equal(hout[s], ref[s]) if s in subset else not hout[s].any(), s
        # in place: row 0 writes block 16 (an input of row 1), row 1 writes block 0 (an input of row 0)
        S, B = 6, 65536
        d = torch.empty((S, 32, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(d, 33)
        h0 = d.cpu().numpy()
        cf = [[1 if (j < 16) == (r == 0) else 0 for j in range(32)] for r in range(2)]
        progs = [(cf, list(range(32)), [16, 0])]
        ecg.matrix_apply_batch_multi(progs, d, d)
        torch.cuda.synchronize()
        ref = h0.copy()
        for s in range(S):
            ref[s, 16] = np.bitwise_xor.reduce(h0[s, 0:16], axis=0)
            ref[s, 0] = np.bitwise_xor.reduce(h0[s, 16:32], axis=0)
        assert np.array_equal(d.cpu().numpy(), ref)
    finally:
        ecg.set_option(ecg.ECG_OPT_ROW_SPLIT, saved)


@pytest.mark.parametrize("B,S", [(65536 + 48, 11), ((1 << 20) + 16, 9), (65536, 13), (1 << 20, 7)])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline_encode_decode(ecg, oracle, torch_cuda, pinned, B, S):
    """Host-resident batches, pinned and pageable, through the H2D -> kernel -> D2H pipeline (chunks not
    dividing S; 64 KiB and 1 MiB blocks, with and without padded device slots).  On pageable buffers a
    second host thread issues the output copies (engine.cpp run_host_pipeline)."""
    torch = torch_cuda
    k, m = 10, 4
    n = k + m
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    if pinned:
        stripes = torch.empty((S, n, B), dtype=torch.uint8).pin_memory()
        stripes.numpy()[:] = np.frombuffer(oracle.splitmix_bytes(4, 0, S * n * B), np.uint8).reshape(S, n, B)
        h = stripes.numpy()
    else:
        h = oracle.splitmix_bytes(4, 0, S * n * B).reshape(S, n, B).copy()
        stripes = h
    data_view = stripes[:, :k]
    coding_view = stripes[:, k:]
    ecg.encode_batch_host(k, m, M, data_view, coding_view, chunk_stripes=4)
    for s in range(S):
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, [h[s, j].copy() for j in range(k)], ref, B)
        assert same([h[s, k + i] for i in range(m)], ref), s
    orig = h.copy()
    out = np.zeros((S, 2, B), np.uint8)
    ecg.decode_batch_host(k, m, M, 1, [2, 12], stripes, h_out=out, chunk_stripes=3)
    assert np.array_equal(out[:, 0], orig[:, 2]) and np.array_equal(out[:, 1], orig[:, 12])
    h[:, 5] = 0
    ecg.decode_batch_host(k, m, M, 1, [5], stripes, chunk_stripes=5)  # in place
    assert np.array_equal(h, orig)


@pytest.mark.parametrize("zc", [0, 1 << 22])
def test_host_tier_staging_paths(ecg, oracle, torch_cuda, zc):
    """Host-buffer calls through the pinned staging area with DMA (zc = 0) or zero-copy kernels on the
    mapped staging memory (ECG_OPT_ZEROCOPY_BYTES): encode, decode, wide pointer tables, multi-op plans."""
    saved = ecg.get_option(ecg.ECG_OPT_ZEROCOPY_BYTES)
    ecg.set_option(ecg.ECG_OPT_ZEROCOPY_BYTES, zc)
    try:
        for k, m, B in [(6, 4, 1024), (10, 4, 4099), (130, 3, 256), (12, 4, 65536)]:
            M = oracle.reed_sol_vandermonde_coding_matrix(k, m) if k + m <= 256 else None
            data = [rnd(B, 7 * j + B) for j in range(k)]
            a = [np.zeros(B, np.uint8) for _ in range(m)]
            b = [np.full(B, 0x33, np.uint8) for _ in range(m)]
            oracle.jerasure_matrix_encode(k, m, M, data, a, B)
            ecg.jerasure_matrix_encode(k, m, M, data, b, B)
            assert same(a, b), (k, m, B)
            if k <= 12:
                stripe = [x.copy() for x in data + a]
                for e in (0, k - 1, k):
                    S = [x.copy() for x in stripe]
                    S[e][:] = 0
                    assert ecg.jerasure_matrix_decode(k, m, M, 1, [e, -1], S[:k], S[k:], B) == 0
                    assert same(S, stripe), (k, e)
        # a product code decode runs several dependent ops in one host call
        o, p = _pair(7, dict(k1=4, m1=1, k2=4, m2=1))
        from oracle import ec_ref as E
        B = 2048
        data = E.blocks(16, B, 5)
        coding = E.zeros(9, B)
        o.encode(data, coding, B)
        D = [x.copy() for x in data]
        C = [x.copy() for x in coding]
        for bid in (0, 1, 5):
            (D[bid] if bid < 16 else C[bid - 16])[:] = 0
        er = [0, 1, 5, -1]
        assert p.decode(D, C, B, er, 3) == 0
        assert same(D, data) and same(C, coding)
    finally:
        ecg.set_option(ecg.ECG_OPT_ZEROCOPY_BYTES, saved)


def test_zero_copy_completion_flags_back_to_back(ecg, oracle, torch_cuda):
    """Zero-copy host calls complete by polled flags, never by a stream synchronize (engine.cpp
    wait_flags): 1500 back-to-back calls on fresh data, each result read right after its flags, cycling
    through flagged shapes (1 KiB, 64 KiB: 32 workgroups, a 2-op decode) and ones that synchronize
    instead (B % 16 != 0: the byte kernel posts no flags), so a stale flag or an early read would show as
    a wrong byte.  More than 64 flagged calls, so the periodic stream query runs too."""
    k, m = 6, 4
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(0xF1A6)
    for i in range(1500):
        B = (1024, 1000, 65536, 1024, 4096 + 48)[i % 5]
        data = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(k)]
        got = [np.full(B, 0x5A, np.uint8) for _ in range(m)]
        assert ecg.jerasure_matrix_encode(k, m, M, data, got, B) == 0
        want = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, data, want, B)
        assert same(got, want), (i, B)
        if i % 50 == 0:  # two erasures: one composed decode op per call
            stripe = [x.copy() for x in data + want]
            S = [x.copy() for x in stripe]
            S[1][:] = 0
            S[k + 2][:] = 0
            assert ecg.jerasure_matrix_decode(k, m, M, 1, [1, k + 2, -1], S[:k], S[k:], B) == 0
            assert same(S, stripe), (i, B)


def test_tuning_options_never_change_results(ecg, oracle, torch_cuda):
    """Every ECG_OPT_* setting (grid map incl. auto, map-2 stripe groups, NT policy, chunk size) gives
    identical bytes, for an in-stripe encode, a separate-buffer decode and S values that do / do not
    divide by 8 (and by 8 G: G = 3 falls back to 1, G = 4 runs as is at S = 32)."""
    torch = torch_cuda
    k, m, B = 10, 4, 3 * 8192 + 16
    n = k + m
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    saved = [ecg.get_option(o) for o in range(ecg.ECG_OPT_COUNT)]
    try:
        for S in (32, 13):
            stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
            ecg.fill_random(stripes, 21 + S)
            ref_par, ref_dec = None, None
            pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
            maps = ((0, 1), (1, 1), (2, 1), (2, 2), (2, 3), (2, 4), (3, 1))
            for (gmap, grp), nt, cpw in itertools.product(maps, (0, 3), (0, 256)):
                ecg.set_option(ecg.ECG_OPT_GRID_MAP, gmap)
                ecg.set_option(ecg.ECG_OPT_MAP_GROUP, grp)
                ecg.set_option(ecg.ECG_OPT_NT, nt)
                ecg.set_option(ecg.ECG_OPT_COLS_PER_WG, cpw)
                stripes[:, k:].fill_(0xA5)
                ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])
                out = torch.full((S, 1, B), 0x3C, dtype=torch.uint8, device="cuda")
                ecg.decode_batch(k, m, M, 1, [[e] for e in range(n)], stripes, out=out, pattern_of_stripe=pos)
                torch.cuda.synchronize()
                if ref_par is None:
                    ref_par, ref_dec = stripes[:, k:].clone(), out.clone()
                    h = stripes.cpu().numpy()
                    for s in (0, S - 1):
                        par = [np.zeros(B, np.uint8) for _ in range(m)]
                        oracle.jerasure_matrix_encode(k, m, M, [h[s, j] for j in range(k)], par, B)
                        assert same([h[s, k + i] for i in range(m)], par)
                    for s in range(S):
                        assert torch.equal(out[s, 0], stripes[s, s % n])
                assert torch.equal(stripes[:, k:], ref_par), (S, gmap, grp, nt, cpw)
                assert torch.equal(out, ref_dec), (S, gmap, grp, nt, cpw)
    finally:
        for o, v in enumerate(saved):
            ecg.set_option(o, v)


@pytest.mark.parametrize("k_in", [2, 4, 6, 8, 10, 16])
def test_mt1_lds_pad_never_changes_results(ecg, oracle, torch_cuda, k_in):
    """ECG_OPT_MT1_LDS_PAD (unused dynamic LDS on single-output vector launches, a cap on workgroups per CU):
    auto (by input count), none, and fixed pads up to the 64 KiB limit give identical bytes for strided
    BINARY and GENERAL k -> 1 launches and a pointer-table scope flush, equal to the oracle's."""
    torch = torch_cuda
    S, B = 24, 8192 + 16
    saved = ecg.get_option(ecg.ECG_OPT_MT1_LDS_PAD)
    d_in = torch.empty((S, k_in, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(d_in, 700 + k_in)
    h = d_in.cpu().numpy()
    rows = {"binary": [1] * k_in, "general": [(11 * j + 5) % 255 + 1 for j in range(k_in)]}
    want = {}
    for name, row in rows.items():
        w = []
        for s in (0, S - 1):
            o = [np.zeros(B, np.uint8)]
            oracle.jerasure_matrix_encode(k_in, 1, row, [h[s, j] for j in range(k_in)], o, B)
            w.append(o[0])
        want[name] = w
    try:
        ref = {}
        for pad in (-1, 0, 12288, 24576, 65536):
            ecg.set_option(ecg.ECG_OPT_MT1_LDS_PAD, pad)
            for name, row in rows.items():
                out = torch.full((S, 1, B), 0x3C, dtype=torch.uint8, device="cuda")
                ecg.matrix_apply_batch(row, list(range(k_in)), [0], d_in, out)
                torch.cuda.synchronize()
                assert np.array_equal(out[0, 0].cpu().numpy(), want[name][0]), (pad, name)
                assert np.array_equal(out[S - 1, 0].cpu().numpy(), want[name][1]), (pad, name)
                ref.setdefault(name, out.clone())
                assert torch.equal(out, ref[name]), (pad, name)
            # the same general row as per-stripe calls in a batch scope: one pointer-table launch
            out = torch.full((S, 1, B), 0x3C, dtype=torch.uint8, device="cuda")
            with ecg.batch():
                for s in range(S):
                    ecg.matrix_apply_batch(rows["general"], list(range(k_in)), [0], d_in[s:s + 1], out[s:s + 1])
            torch.cuda.synchronize()
            assert torch.equal(out, ref["general"]), (pad, "scope")
    finally:
        ecg.set_option(ecg.ECG_OPT_MT1_LDS_PAD, saved)


# ------------------------------------------------------------------ edge sizes: the GF(2^8) field limit, empty inputs

@pytest.mark.parametrize("k,m", [(250, 6), (200, 56), (128, 128), (255, 1), (1, 255)])
def test_max_field_rs_encode_decode(ecg, oracle, torch_cuda, k, m):
    """k + m = 256, the largest stripe reed_sol_vandermonde_coding_matrix allows at w = 8: pointer-table
    launches (k > 128 inputs or m > 32 outputs), up to 32 row tiles, decode with exactly m erasures
    (a k x k inverse of up to 255 x 255 on the host), B with a byte tail."""
    torch = torch_cuda
    B = 4099
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    assert ecg.reed_sol_vandermonde_coding_matrix(k, m) == M
    assert ecg.reed_sol_vandermonde_coding_matrix(k, m + 1) is None  # k + m + 1 = 257 > 2^w
    data = [rnd(B, 7 * j + k) for j in range(k)]
    a = [np.zeros(B, np.uint8) for _ in range(m)]
    b = [np.full(B, 0xA5, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data, a, B)
    ecg.jerasure_matrix_encode(k, m, M, data, b, B)
    assert same(a, b)
    stripe = data + a
    rng = random.Random(k * 1000 + m)
    for pat in (rng.sample(range(k + m), m), list(range(k + m - m, k + m)), rng.sample(range(k + m), max(1, m // 2))):
        A = [x.copy() for x in stripe]
        Bb = [x.copy() for x in stripe]
        for i in pat:
            A[i][:] = 0xEE
            Bb[i][:] = 0xEE
        ra = oracle.jerasure_matrix_decode(k, m, M, 1, pat + [-1], A[:k], A[k:], B)
        rb = ecg.jerasure_matrix_decode(k, m, M, 1, pat + [-1], Bb[:k], Bb[k:], B)
        assert ra == rb == 0, pat
        assert same(A, Bb) and same(A, stripe), pat
    # m + 1 erasures: undecodable, -1 like the library, buffers untouched
    pat = rng.sample(range(k + m), min(k + m, m + 1))
    if len(pat) == m + 1:
        A = [x.copy() for x in stripe]
        assert ecg.jerasure_matrix_decode(k, m, M, 1, pat + [-1], A[:k], A[k:], B) == -1
        assert same(A, stripe)
    # batched device tier at the same size: [S][k+m][B'] with B' = 4 KiB + 16
    S, Bd = 3, 4096 + 16
    st = torch.empty((S, k + m, Bd), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 0xF1E1D + k)
    ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])
    host = st.cpu().numpy()
    for s in range(S):
        ref_c = [np.zeros(Bd, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, [host[s, j] for j in range(k)], ref_c, Bd)
        assert all(np.array_equal(ref_c[i], host[s, k + i]) for i in range(m)), s


@pytest.mark.parametrize("k,m", [(200, 56), (100, 4)])
def test_max_field_cauchy_good(ecg, oracle, torch_cuda, k, m):
    B = 1000
    C = oracle.cauchy_good_general_coding_matrix(k, m)
    assert ecg.cauchy_good_general_coding_matrix(k, m) == C
    data = [rnd(B, 3 * j + m) for j in range(k)]
    a = [np.zeros(B, np.uint8) for _ in range(m)]
    b = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, C, data, a, B)
    ecg.jerasure_matrix_encode(k, m, C, data, b, B)
    assert same(a, b)


def test_empty_inputs(ecg, oracle, torch_cuda):
    """B = 0 and S = 0 are no-ops that return 0 and touch nothing; negative sizes are ECG_EINVAL."""
    torch = torch_cuda
    k, m = 10, 4
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    e0 = np.zeros(0, np.uint8)
    ecg.jerasure_matrix_encode(k, m, M, [e0] * k, [e0.copy() for _ in range(m)], 0)
    assert ecg.jerasure_matrix_decode(k, m, M, 1, [0, -1], [e0] * k, [e0.copy() for _ in range(m)], 0) == 0
    guard = torch.full((2, k + m, 64), 7, dtype=torch.uint8, device="cuda")
    ecg.encode_batch(k, m, M, guard[:0, :k], guard[:0, k:])                        # S = 0
    ecg.encode_batch(k, m, M, guard[:, :k, :0], guard[:, k:, :0])                   # B = 0
    ecg.decode_batch(k, m, M, 1, [[3]], guard[:0])
    ecg.perform_addition_batch(2, 1, guard[:0, :2], guard[:0, 2:3])
    ecg.matrix_apply_batch([[1, 1]], [0, 1], [0], guard[:0, :2], guard[:0, 2:3])
    h = np.zeros((0, k + m, 64), np.uint8)
    ecg.encode_batch_host(k, m, M, h[:, :k], h[:, k:])
    torch.cuda.synchronize()
    assert bool((guard == 7).all())
    L = ecg.lib()
    rc = L.ecg_encode_batch(k, m, ecg._ints(M), guard.data_ptr(), guard.stride(0), guard.stride(1),
                            guard.data_ptr() + k * 64, guard.stride(0), guard.stride(1), 64, -1, None)
    assert rc == ecg.ECG_EINVAL
    rc = L.ecg_encode_batch(k, m, ecg._ints(M), guard.data_ptr(), guard.stride(0), guard.stride(1),
                            guard.data_ptr() + k * 64, guard.stride(0), guard.stride(1), -5, 2, None)
    assert rc == ecg.ECG_EINVAL
    torch.cuda.synchronize()
    assert bool((guard == 7).all())


# ------------------------------------------------------------------ deferred-batch scope (ecg_batch_begin / _end)

def test_batch_scope_per_stripe_calls(ecg, oracle, torch_cuda):
    """Per-stripe ErasureCode calls on HBM buffers inside a batch scope (the reference's one-call-per-
    stripe loop, proxy.cpp:312-349) give the same bytes as the batched tier, and nothing is launched
    before the scope ends."""
    torch = torch_cuda
    k, m, S, B = 10, 4, 48, 64 * 1024 + 16
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    st = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 0xBA7C4)
    ref = st.clone()
    ecg.encode_batch(k, m, M, ref[:, :k], ref[:, k:])
    st[:, k:] = 0x5A
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))
    with ecg.batch() as scope:
        for s in range(S // 2):
            ec.encode([st[s, j] for j in range(k)], [st[s, k + i] for i in range(m)], B)
        torch.cuda.synchronize()
        assert bool((st[:, k:] == 0x5A).all()), "deferred calls ran before the scope ended"
        scope.flush()  # ecg_batch_flush: the recorded half is launched, the scope stays open
        torch.cuda.synchronize()
        assert torch.equal(st[:S // 2], ref[:S // 2])
        for s in range(S // 2, S):
            ec.encode([st[s, j] for j in range(k)], [st[s, k + i] for i in range(m)], B)
        torch.cuda.synchronize()
        assert bool((st[S // 2:, k:] == 0x5A).all()), "deferred calls ran before the scope ended"
    torch.cuda.synchronize()
    assert torch.equal(st, ref)
    # decode: runs of 8 stripes share an erasure pattern (one batched launch per run)
    lost = torch.empty((S, 2, B), dtype=torch.uint8, device="cuda")
    pats = [[(s // 8) % n, (s // 8 + 5) % n] for s in range(S)]
    for s in range(S):
        for e in pats[s]:
            st[s, e] = 0xEE
    with ecg.batch():
        for s in range(S):
            ec.decode([st[s, j] for j in range(k)], [st[s, k + i] for i in range(m)], B, pats[s] + [-1], 2)
    torch.cuda.synchronize()
    assert torch.equal(st, ref)
    host = ref[:3].cpu().numpy()
    for s in range(3):
        coding = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, [host[s, j] for j in range(k)], coding, B)
        assert all(np.array_equal(coding[i], host[s, k + i]) for i in range(m))


@pytest.mark.parametrize("with_scratch", [False, True])
def test_batch_scope_eager_flush(ecg, torch_cuda, with_scratch):
    """Without declared scratch the scope flushes by itself every 1024 recorded calls (the GPU works while
    the host records); with scratch it keeps recording up to 65536.  3000 calls -- an encode per stripe,
    then a perform_addition per stripe reading that stripe's parities -- cross the 1024 boundaries with
    dependences on both sides, and give the bytes of the same calls made outside any scope."""
    torch = torch_cuda
    k, m, S, B = 4, 2, 1500, 256 + 16
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    st = torch.empty((S, k + m, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 0xEA6E)
    st[:, k:] = 0x5A
    out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
    ref_st, ref_out = st.clone(), out.clone()
    dummy = torch.empty(4096, dtype=torch.uint8, device="cuda")
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))

    def calls(x, o):
        for s in range(S):
            ec.encode([x[s, j] for j in range(k)], [x[s, k + i] for i in range(m)], B)
        for s in range(S):
            ec.perform_addition([x[s, k], x[s, k + 1]], [o[s]], B, 2, 1)

    calls(ref_st, ref_out)
    with ecg.batch() as scope:
        if with_scratch:
            scope.scratch(dummy)  # unrelated scratch: nothing composes, but no eager flush either
        calls(st, out)
    torch.cuda.synchronize()
    assert torch.equal(st, ref_st) and torch.equal(out, ref_out)
    assert bool((out == (st[:, k] ^ st[:, k + 1])).all())
    stats = ecg.batch_last_stats()
    assert stats["recorded"] == (2 * S if with_scratch else (2 * S) % 1024), stats


@pytest.mark.parametrize("a_null", [False, True], ids=["a_created", "a_null_stream"])
def test_batch_scope_orders_streams(ecg, torch_cuda, a_null):
    """Calls recorded on two streams in one scope keep their recorded order: the flush makes a
    group wait for an event behind the previous group where the stream changes.  Stream A encodes a large
    batch; stream B then adds each stripe's first two parities (reads A's output); and a helper partial
    recorded on A into declared scratch is consumed by a perform_addition recorded on B (the composed op
    runs on B and must see A's encode).  Without the ordering, B's kernels race A's.  A is also torch's
    default stream -- the null stream, handle 0, which the flush once took for "no previous group"."""
    torch = torch_cuda
    k, m, S, B = 10, 4, 256, 1 << 20
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    st = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 0x0D3D)
    st[:, k:] = 0
    out = torch.zeros((S, 2, B), dtype=torch.uint8, device="cuda")
    scratch = torch.empty((S, B), dtype=torch.uint8, device="cuda")
    ref = st.clone()
    ecg.encode_batch(k, m, M, ref[:, :k], ref[:, k:])
    want0 = ref[:, k] ^ ref[:, k + 1]
    want1 = ref[:, k + 2] ^ ref[:, k + 3] ^ ref[:, 0]
    torch.cuda.synchronize()
    # B at high priority: a hardware queue of its own (two streams sharing one would run in order anyway)
    sa = torch.cuda.default_stream() if a_null else torch.cuda.Stream()
    sb = torch.cuda.Stream(priority=-1)
    assert (sa.cuda_stream == 0) == a_null
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))
    for _ in range(2):
        out.zero_()
        st[:, k:] = 0
        torch.cuda.synchronize()
        with ecg.batch() as scope:
            scope.scratch(scratch)
            for s in range(S):
                ec.encode([st[s, j] for j in range(k)], [st[s, k + i] for i in range(m)], B, stream=sa.cuda_stream)
            for s in range(S):
                ec.perform_addition([st[s, k], st[s, k + 1]], [out[s, 0]], B, 2, 1, stream=sb.cuda_stream)
            for s in range(S):  # scratch partial on A, consumed on B
                ec.perform_addition([st[s, k + 2], st[s, k + 3]], [scratch[s]], B, 2, 1, stream=sa.cuda_stream)
                ec.perform_addition([scratch[s], st[s, 0]], [out[s, 1]], B, 2, 1, stream=sb.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(st, ref)
        assert torch.equal(out[:, 0], want0), "stream B read parities before stream A wrote them"
        assert torch.equal(out[:, 1], want1), "composed op on stream B did not see stream A's encode"


def test_batch_scope_orders_streams_across_eager_flushes(ecg, torch_cuda):
    """A scope without scratch flushes by itself every 1024 recorded calls, so a dependence can straddle two
    flushes: 1024 encodes recorded on stream A fill the first flush, and the next flush starts with stream
    B's additions of their parities.  B's first group must still wait for A (the scope keeps program order
    across its flushes, not only inside one).  Stream A is kept busy beforehand, so B's kernels would run
    long before A's encodes if they did not wait."""
    torch = torch_cuda
    k, m, S, B = 10, 4, 1024, 64 << 10
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    st = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 0x0E7F)
    ref = st.clone()
    ecg.encode_batch(k, m, M, ref[:, :k], ref[:, k:])
    want = ref[:, k] ^ ref[:, k + 1]
    busy = torch.empty((512, n, 1 << 20), dtype=torch.uint8, device="cuda")  # 7 GiB of stripes
    # B at high priority: HIP maps streams onto a few hardware queues, and two streams that share one run in
    # queue order anyway, which would hide a missing wait; a high-priority stream has a queue of its own
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream(priority=-1)
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))
    out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        out.zero_()
        st[:, k:] = 0
        torch.cuda.synchronize()
        for _ in range(100):  # ~120 ms of encodes queued on A ahead of the scope's calls
            ecg.encode_batch(k, m, M, busy[:, :k], busy[:, k:], stream=sa.cuda_stream)
        with ecg.batch():
            for s in range(S):  # exactly one eager flush's worth, all on A
                ec.encode([st[s, j] for j in range(k)], [st[s, k + i] for i in range(m)], B, stream=sa.cuda_stream)
            for s in range(S):  # the next flush opens with B
                ec.perform_addition([st[s, k], st[s, k + 1]], [out[s]], B, 2, 1, stream=sb.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(st, ref)
        assert torch.equal(out, want), "stream B's first group of a flush ran before stream A's previous flush"


def test_batch_scope_strided_fast_path_and_sliding_windows(ecg, torch_cuda):
    """A flush whose calls share one plan and form one overlap-free strided batch takes one group without
    the hazard hash (the per-stripe loop over [S][n][B] and over block-major [n][S][B]); a strided run whose
    calls overlap -- a sliding window, call c encoding blocks c .. c+9 into c+10 .. c+13, every call
    reading its predecessors' parities -- must not, and gives the sequential bytes."""
    torch = torch_cuda
    k, m, B = 10, 4, 4096
    n = k + m
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))
    for layout in ("stripe-major", "block-major"):
        S = 300
        buf = torch.empty((S, n, B) if layout == "stripe-major" else (n, S, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(buf, 0x5EED)
        st = buf if layout == "stripe-major" else buf.permute(1, 0, 2)
        ref = st.clone()
        M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
        ecg.encode_batch(k, m, M, ref[:, :k], ref[:, k:])
        with ecg.batch():
            for s_ in range(S):
                ec.encode([st[s_, j] for j in range(k)], [st[s_, k + i] for i in range(m)], B)
        torch.cuda.synchronize()
        assert torch.equal(st, ref), layout
        assert ecg.batch_last_stats()["launches"] == 1, (layout, ecg.batch_last_stats())  # one group, one op
    # sliding windows over one row of blocks: strided (stripe stride = one block) but overlapping
    S = 200
    row = torch.empty((S + n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(row, 0x51DE)
    want = row.clone()
    for s_ in range(S):  # outside any scope: the sequential bytes
        ec.encode([want[s_ + j] for j in range(k)], [want[s_ + k + i] for i in range(m)], B)
    with ecg.batch():
        for s_ in range(S):
            ec.encode([row[s_ + j] for j in range(k)], [row[s_ + k + i] for i in range(m)], B)
    torch.cuda.synchronize()
    assert torch.equal(row, want), "sliding-window calls must keep their order"
    assert ecg.batch_last_stats()["launches"] > 1


def test_batch_scope_hazards_split_runs(ecg, torch_cuda):
    """Calls with the same plan that depend on each other (a chain of galois_region_xor-like additions
    through perform_addition) must keep their sequential meaning inside a scope."""
    torch = torch_cuda
    B, N = 4096 + 7, 12
    bufs = torch.randint(0, 256, (N + 1, B), dtype=torch.uint8, device="cuda")
    expect = bufs.cpu().numpy().copy()
    for i in range(1, N + 1):
        expect[i] ^= expect[i - 1]  # acc_i = in_i ^ acc_{i-1}, sequentially
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=4, m=2))
    with ecg.batch():
        for i in range(1, N + 1):
            ec.perform_addition([bufs[i - 1], bufs[i]], [bufs[i]], B, 2, 1)
    torch.cuda.synchronize()
    assert np.array_equal(bufs.cpu().numpy(), expect)
    # independent calls of the same plan, interleaved with a host-tier call (which flushes first)
    a = torch.randint(0, 256, (6, B), dtype=torch.uint8, device="cuda")
    out = torch.zeros((3, B), dtype=torch.uint8, device="cuda")
    h_src, h_dst = np.full(B, 3, np.uint8), np.full(B, 5, np.uint8)
    with ecg.batch():
        for i in range(3):
            ec.perform_addition([a[2 * i], a[2 * i + 1]], [out[i]], B, 2, 1)
        ecg.galois_region_xor(h_src, h_dst, B)
        torch.cuda.synchronize()
        assert torch.equal(out, a[0::2] ^ a[1::2])  # flushed by the host-tier call
        with pytest.raises(ecg.EcgError):
            ecg.batch().__enter__()  # scopes do not nest
    assert (h_dst == 6).all()


def test_batch_scope_then_direct_batched_calls(ecg, oracle, torch_cuda):
    """Batched entry points that launch directly flush the scope's recorded calls first, whatever launch
    they pick: region_xor_batch with S = 1 and with unaligned strides (pointer-table launch), and
    fill_random.  Without the flush they would run before the recorded encode they depend on."""
    torch = torch_cuda
    k, m, B = 4, 2, 4096
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))
    st = torch.empty((3, k + m, B + 4), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 77)
    host = st.cpu().numpy()
    want = []
    for s in range(3):
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, [host[s, j, :B].copy() for j in range(k)], ref, B)
        want.append(ref)
    acc = torch.zeros((B,), dtype=torch.uint8, device="cuda")
    with ecg.batch():
        ec.encode([st[0, j, :B] for j in range(k)], [st[0, k + i, :B] for i in range(m)], B)
        ecg.region_xor_batch(st[0, k, :B].reshape(1, B), acc.reshape(1, B))  # S = 1: pointer-table launch
    torch.cuda.synchronize()
    assert np.array_equal(acc.cpu().numpy(), want[0][0])
    # unaligned strides (B + 4): not a strided launch either
    acc2 = torch.zeros((2, B + 4), dtype=torch.uint8, device="cuda")
    with ecg.batch():
        for s in (1, 2):
            ec.encode([st[s, j, :B] for j in range(k)], [st[s, k + i, :B] for i in range(m)], B)
        ecg.region_xor_batch(st[1:, k + 1, :B], acc2[:, :B])
    torch.cuda.synchronize()
    for s in (1, 2):
        assert np.array_equal(acc2[s - 1, :B].cpu().numpy(), want[s][1]), s
    # fill_random after a recorded encode that reads the filled block: the encode sees the old bytes
    blk = torch.empty((k + m, B), dtype=torch.uint8, device="cuda")
    blk[:k].copy_(st[0, :k, :B])
    with ecg.batch():
        ec.encode([blk[j] for j in range(k)], [blk[k + i] for i in range(m)], B)
        ecg.fill_random(blk[0], 99)
    torch.cuda.synchronize()
    assert same([blk[k + i].cpu().numpy() for i in range(m)], want[0])


def test_batch_scope_flush_on_recording_device(ecg, torch_cuda):
    """Calls recorded on device 0 and flushed after the thread switched to device 1 launch on device 0
    (needs two GPUs; the pool's boxes have one)."""
    torch = torch_cuda
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=4, m=2))
    a = torch.randint(0, 256, (6, 4096), dtype=torch.uint8, device="cuda:0")
    ref = a.clone()
    ecg.encode_batch(4, 2, ecg.reed_sol_vandermonde_coding_matrix(4, 2), ref[None, :4], ref[None, 4:])
    a[4:] = 0
    torch.cuda.set_device(0)
    ecg.lib().ecg_set_device(0)
    with ecg.batch():
        ec.encode([a[j] for j in range(4)], [a[4 + i] for i in range(2)], 4096)
        ecg.lib().ecg_set_device(1)
    ecg.lib().ecg_set_device(0)
    torch.cuda.synchronize(0)
    assert torch.equal(a, ref)


def _azure_repair_state(ecg, torch, S, B, seed):
    """Azure-LRC(12,2,2) stripes [S][16][B] on the GPU, block e = s mod 14 of stripe s lost (local repairs:
    data and local parities), with the helper / main split of handle_repair.cpp."""
    from ecg_ring import azure_local_split
    k, l, g = 12, 2, 2
    cp = ecg.CodingParameters(k=k, l=l, g=g, local_or_column=True)
    ec = ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    st = torch.empty((S, k + g + l, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, seed)
    ecg.encode_batch(k, g + l, ec.make_encoding_matrix(), st[:, :k], st[:, k:])
    local = [e for e in range(16) if e not in (12, 13)]
    plan = [(local[s % len(local)],) + azure_local_split(local[s % len(local)]) for s in range(S)]
    return ec, st, plan


def _repair_sequence(ec, st, plan, partials, out, B):
    """The reference's partial-decoding repair of every stripe, call by call (handle_repair.cpp:249,
    371-376): helper partial, main partial, perform_addition of the two."""
    for s, (e, surv, sets) in enumerate(plan):
        for i in range(2):
            ec.encode_partial_blocks_for_decoding([st[s, b] for b in sets[i]], [partials[s, i]], B, sets[i], surv, [e])
        ec.perform_addition([partials[s, 0], partials[s, 1]], [out[s]], B, 2, 1)


def test_batch_scope_interleaved_plans_group(ecg, torch_cuda):
    """Per-stripe repairs interleave three plans per stripe and a different erasure per stripe; the scope
    still launches one launch per distinct plan SHAPE (single-op plans of one shape share a multi-program
    pointer-table launch; calls reordered where nothing orders them), and the bytes are the sequential ones."""
    torch = torch_cuda
    S, B = 56, 64 * 1024
    ec, st, plan = _azure_repair_state(ecg, torch, S, B, 0x5C0)
    partials = torch.zeros((S, 2, B), dtype=torch.uint8, device="cuda")
    out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
    with ecg.batch():
        _repair_sequence(ec, st, plan, partials, out, B)
    torch.cuda.synchronize()
    stats = ecg.batch_last_stats()
    idx = torch.arange(S, device="cuda")
    want = st[idx, torch.tensor([p[0] for p in plan], device="cuda")]
    assert torch.equal(out, want)
    assert stats["recorded"] == 3 * S and stats["composed"] == 3 * S
    # one launch per distinct (k_in, m_out) of the partial plans -- whatever their matrices -- + the
    # perform_addition plan, which reads the partials
    shapes = {(len(sets[i]), 1) for e, surv, sets in plan for i in range(2)}
    assert stats["launches"] == len(shapes) + 1, (stats, shapes)


def test_batch_scope_scratch_composes_partials(ecg, oracle, torch_cuda):
    """batch_scratch on the partial buffers: the helper partial + main partial + perform_addition of
    every stripe compose into ONE region product per repair (7 block moves instead of 11), the partial
    buffers are never written, and the repaired blocks equal the lost ones (and the oracle's repair)."""
    torch = torch_cuda
    S, B = 56, 64 * 1024 + 16  # + 16: byte-path tails too
    ec, st, plan = _azure_repair_state(ecg, torch, S, B, 0x5C1)
    partials = torch.full((S, 2, B), 0xA5, dtype=torch.uint8, device="cuda")
    out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
    with ecg.batch() as scope:
        scope.scratch(partials)
        _repair_sequence(ec, st, plan, partials, out, B)
    torch.cuda.synchronize()
    stats = ecg.batch_last_stats()
    idx = torch.arange(S, device="cuda")
    want = st[idx, torch.tensor([p[0] for p in plan], device="cuda")]
    assert torch.equal(out, want)
    assert bool((partials == 0xA5).all()), "scratch partials were written"
    composed = {tuple(ec.partial_decoding_matrix(surv, surv, [e])) for e, surv, _ in plan}
    assert stats == {"recorded": 3 * S, "composed": S, "launches": len(composed), "materialised": 0}, stats
    # the composed map of one stripe is the oracle's full local repair of that block
    host = st[:2].cpu().numpy()
    for s in range(2):
        e, surv, _ = plan[s]
        R = ec.partial_decoding_matrix(surv, surv, [e])
        rebuilt = np.zeros(B, np.uint8)
        oracle.jerasure_matrix_encode(len(surv), 1, list(R), [host[s, b] for b in surv], [rebuilt], B)
        assert np.array_equal(rebuilt, out[s].cpu().numpy())


def test_batch_scope_scratch_mid_scope_flush_and_streams(ecg, torch_cuda):
    """A scratch partial still pending at a mid-scope flush is written for real (memory as if the calls
    ran one by one); one read on another stream is written for real before that read; one never read is
    not written at scope end."""
    torch = torch_cuda
    S, B = 8, 4096
    ec, st, plan = _azure_repair_state(ecg, torch, S, B, 0x5C2)
    partials = torch.full((S, 2, B), 0x3C, dtype=torch.uint8, device="cuda")
    out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
    ref_p = torch.zeros_like(partials)
    ref_o = torch.zeros_like(out)
    _repair_sequence(ec, st, plan, ref_p, ref_o, B)  # outside any scope: the sequential bytes
    torch.cuda.synchronize()
    with ecg.batch() as scope:
        scope.scratch(partials)
        for s, (e, surv, sets) in enumerate(plan):
            for i in range(2):
                ec.encode_partial_blocks_for_decoding([st[s, b] for b in sets[i]], [partials[s, i]], B, sets[i], surv, [e])
        scope.flush()
        torch.cuda.synchronize()
        assert torch.equal(partials, ref_p), "mid-scope flush must write pending scratch"
        assert ecg.batch_last_stats()["materialised"] == 2 * S
    # another stream reads a scratch partial: written for real first, on the producer's stream (torch's
    # default stream, the null stream: the side read must wait for it -- it raced it in 1 run of 3 before
    # the flush stopped taking handle 0 for "no previous group"; a few trials make such a race show)
    side = torch.cuda.Stream(priority=-1)  # a hardware queue of its own: a missing wait would show
    for trial in range(12):
        partials.fill_(0x3C)
        out.zero_()
        torch.cuda.synchronize()
        with ecg.batch() as scope:
            scope.scratch(partials)
            for s, (e, surv, sets) in enumerate(plan):
                for i in range(2):
                    ec.encode_partial_blocks_for_decoding([st[s, b] for b in sets[i]], [partials[s, i]], B, sets[i], surv, [e])
            ec.perform_addition([partials[0, 0], partials[0, 1]], [out[0]], B, 2, 1, stream=side.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(out[0], ref_o[0]), f"trial {trial}: side-stream read raced the write-out"
        assert torch.equal(partials[0], ref_p[0])
        assert bool((partials[1:] == 0x3C).all()), "unconsumed scratch must not be written at scope end"


def test_batch_scope_random_sequences(ecg, torch_cuda):
    """Random per-call region products (dev_matrix_encode over blocks drawn from a small pool, so calls
    depend on each other, some blocks scratch) inside a scope, against the same calls run one by one
    outside any scope; non-scratch blocks must match exactly."""
    torch = torch_cuda
    rng = random.Random(0xF00D)
    B, P = 256, 12
    for trial in range(30):
        pool0 = torch.randint(0, 256, (P, B), dtype=torch.uint8, device="cuda")
        scratch = [b for b in range(P) if rng.random() < 0.3]
        calls = []
        for _ in range(rng.randint(1, 40)):
            k, m = rng.randint(1, 4), rng.randint(1, 3)
            ids = rng.sample(range(P), k + m) if rng.random() < 0.8 else [rng.randrange(P) for _ in range(k + m)]
            M = [rng.choice([0, 1, 1, rng.randrange(256)]) for _ in range(k * m)]
            calls.append((k, m, M, ids))

        def run(pool):
            for k, m, M, ids in calls:
                ecg.dev_matrix_encode(k, m, M, [pool[i] for i in ids[:k]], [pool[i] for i in ids[k:]], B)

        seq = pool0.clone()
        run(seq)
        got = pool0.clone()
        with ecg.batch() as scope:
            for b in scratch:
                scope.scratch(got[b])
            run(got)
        torch.cuda.synchronize()
        keep = [b for b in range(P) if b not in scratch]
        assert torch.equal(got[keep], seq[keep]), (trial, calls, scratch)


# ------------------------------------------------------------------ randomized code parameters, every family

def _random_configs(n, seed):
    """Random valid parameters for every ECTYPE (divisibility kept so groups are whole; Cauchy LRCs with
    g >= 2 since g = 1 needs the unpinned cbest_8 table)."""
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        t = rng.randrange(10)
        if t == 0:
            p = dict(k=rng.randint(1, 40), m=rng.randint(1, 8))
        elif t == 1:
            x = rng.randint(2, 4)
            p = dict(k=rng.randint(2, 12), m=rng.randint(1, 4), x=x, seri_num=rng.randrange(x))
        elif t in (2, 5):  # Azure, Optimal-Cauchy: l | k
            l = rng.randint(1, 4)
            p = dict(k=l * rng.randint(2, 6), l=l, g=rng.randint(2 if t == 5 else 1, 4))
        elif t == 3:       # Azure+1: (l - 1) | k
            l = rng.randint(2, 4)
            p = dict(k=(l - 1) * rng.randint(2, 6), l=l, g=rng.randint(1, 3))
        elif t in (4, 6):  # Optimal, Uniform-Cauchy: l | (k + g)
            l = rng.randint(1, 4)
            g = rng.randint(2 if t == 6 else 1, 4)
            kg = l * rng.randint(max(2, (g + 2 + l - 1) // l), 6)
            p = dict(k=kg - g, l=l, g=g)
        else:              # PC, HPC, HVPC
            p = dict(k1=rng.randint(2, 5), m1=rng.randint(1, 2), k2=rng.randint(2, 4), m2=rng.randint(1, 2))
            if t == 8:
                p.update(x=rng.randint(2, 3), seri_num=0)
                p["seri_num"] = rng.randrange(p["x"])
        out.append((f"rand{len(out)}-{t}-{p}", t, p))
    return out


@pytest.mark.parametrize("name,t,params", _random_configs(60, 0xC0DE5))
def test_random_codes_vs_oracle(ecg, oracle, torch_cuda, name, t, params):
    """Encode, decode (random patterns, garbage-free erased buffers) and partial encode/decode of
    randomly drawn parameters of every code family, product vs oracle, byte for byte."""
    from oracle import ec_ref as E
    B = 1024 + 3
    o, p = _pair(t, params)
    data = E.blocks(o.k, B, 11)
    ca, cb = E.zeros(o.m, B), E.zeros(o.m, B)
    o.encode(data, ca, B)
    assert p.encode(data, cb, B) == 0
    assert same(ca, cb), name
    test_facade_decode_vs_oracle(ecg, oracle, torch_cuda, name, t, params)
    test_facade_partials_vs_oracle(ecg, oracle, torch_cuda, name, t, params)


def test_program_cache_bounded(ecg, oracle, torch_cuda):
    """More distinct coefficient programs than ECG_OPT_PROGRAM_CACHE: the cache stays bounded (LRU half
    dropped after a device synchronize) and every result stays exact, including launches still in
    flight when their program is evicted."""
    torch = torch_cuda
    saved = ecg.get_option(ecg.ECG_OPT_PROGRAM_CACHE)
    rng = random.Random(77)
    k, m, B = 6, 3, 8192 + 16
    try:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, 8)
        d = torch.empty((40, k + m, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(d, 0xCAC4E)
        mats = [[rng.randrange(256) for _ in range(k * m)] for _ in range(40)]
        for s in range(40):  # asynchronous launches, one new program each
            ecg.encode_batch(k, m, mats[s], d[s:s + 1, :k], d[s:s + 1, k:])
            assert ecg.lib().ecg_program_cache_size() <= 8
        torch.cuda.synchronize()
        host = d.cpu().numpy()
        for s in range(40):
            coding = [np.zeros(B, np.uint8) for _ in range(m)]
            oracle.jerasure_matrix_encode(k, m, mats[s], [host[s, j] for j in range(k)], coding, B)
            assert all(np.array_equal(coding[i], host[s, k + i]) for i in range(m)), s
    finally:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, saved)


def test_large_host_blocks(ecg, oracle, torch_cuda):
    """The reference's SET buffers (proxy.cpp:335-339): k slices of ONE contiguous value buffer and m
    separate parity buffers, 1 MiB blocks, from four threads that share the value buffer as input.  The
    large-block host path (pageable copies, contiguous runs coalesced, the caller's pages never
    registered) returns the oracle's bytes for separate parity buffers, for parities forming one
    odd-offset run inside a shared buffer (its neighbours untouched), and for an in-place decode whose
    outputs are slices next to input slices."""
    k, m, B = 10, 4, (1 << 20) + 5
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    value = rnd(k * B, 4242)
    data = [value[j * B:(j + 1) * B] for j in range(k)]
    expect = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data, expect, B)
    shared = np.full(3 + m * B + 7, 0x77, np.uint8)  # thread 3: parities as one contiguous odd run
    outs = [[np.zeros(B, np.uint8) for _ in range(m)] for _ in range(3)]
    outs.append([shared[3 + i * B:3 + (i + 1) * B] for i in range(m)])
    errs = []

    def work(t):
        try:
            for _ in range(3):
                ecg.jerasure_matrix_encode(k, m, M, data, outs[t], B)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    [x.start() for x in th]
    [x.join() for x in th]
    assert not errs, errs
    for t in range(4):
        assert same(outs[t], expect), t
    assert (shared[:3] == 0x77).all() and (shared[3 + m * B:] == 0x77).all()  # neighbours untouched
    # decode in place: lose data 3 and parity 1 (garbage in both), survivors are slices of `value`
    stripe = data + [x.copy() for x in expect]
    orig = value.copy()
    lost = [stripe[3].copy(), stripe[k + 1].copy()]
    stripe[3][:] = 0xEE
    stripe[k + 1][:] = 0xEE
    assert ecg.jerasure_matrix_decode(k, m, M, 2, [3, k + 1, -1], stripe[:k], stripe[k:], B) == 0
    assert np.array_equal(stripe[3], lost[0]) and np.array_equal(stripe[k + 1], lost[1])
    assert np.array_equal(value, orig)  # the rebuilt slice is exact and its neighbour slices untouched


@pytest.mark.parametrize("aligned", [False, True])
def test_region_xor_batch(ecg, oracle, torch_cuda, aligned):
    """ecg_region_xor_batch: galois_region_xor (dst ^= src) over S regions, any strides / sizes
    (16-byte-multiple strides go out as a strided launch, the others through a pointer table)."""
    torch = torch_cuda
    for S, n in [(1, 1), (7, 1000), (64, 4096 + 3), (3, 1 << 20), (8, 4096), (5, 65536 + 32)]:
        if aligned:
            n = (n + 15) & ~15
            src = torch.randint(0, 256, (S, n), dtype=torch.uint8, device="cuda")
        else:
            src = torch.randint(0, 256, (S, n + 16), dtype=torch.uint8, device="cuda")[:, 5:5 + n]  # odd stride/offset
        dst = torch.randint(0, 256, (S, n), dtype=torch.uint8, device="cuda")
        expect = (src.cpu().numpy() ^ dst.cpu().numpy())
        ecg.region_xor_batch(src, dst)
        torch.cuda.synchronize()
        assert np.array_equal(dst.cpu().numpy(), expect), (S, n)
        a, b = np.frombuffer(bytes(src[0].cpu().numpy()), np.uint8).copy(), dst[0].cpu().numpy().copy()
        c = b.copy()
        oracle.galois_region_xor(a, c, n)  # self-inverse: XOR the source back in
        assert np.array_equal(c, b ^ a)


@pytest.mark.parametrize("isvertical", [True, False])
@pytest.mark.parametrize("seri_num", [0, 1])
def test_hpc_orientation_vs_oracle(ecg, oracle, torch_cuda, isvertical, seri_num):
    """HPC::isvertical (pc.h:65) picks which dimension uses the enlarged RS code (pc.cpp:585-619,
    680-728, 755-835): the merged-stripe orientation of config 4.  Encode, decode and the partial
    encodings / decodings of one row and one column, for both orientations, against the oracle."""
    from oracle import ec_ref as E
    params = dict(k1=4, m1=2, k2=2, m2=1, x=2, seri_num=seri_num)
    cp = E.CodingParameters(**params)
    o = E.ec_factory(8, cp)
    o.init_coding_parameters(cp)
    o.isvertical = isvertical
    p = ecg.ec_factory(8, ecg.CodingParameters(**params))
    p.init_coding_parameters(ecg.CodingParameters(**params))
    p.set_isvertical(isvertical)
    B = 2048 + 7
    rng = random.Random(seri_num * 2 + isvertical)
    data = E.blocks(o.k, B, 11 + seri_num)
    ca, cb = E.zeros(o.m, B), E.zeros(o.m, B)
    o.encode(data, ca, B)
    assert p.encode(data, cb, B) == 0
    assert same(ca, cb), "encode"
    stripe = data + ca
    n = o.k + o.m
    for _ in range(8):
        pat = rng.sample(range(n), rng.randint(1, 3))
        A, Bq = [x.copy() for x in stripe], [x.copy() for x in stripe]
        for i in pat:
            A[i][:] = 0
            Bq[i][:] = 0
        ra = o.decode(A[:o.k], A[o.k:], B, pat + [-1], len(pat))
        rb = p.decode(Bq[:o.k], Bq[o.k:], B, pat + [-1], len(pat))
        assert (ra == 0) == (rb == 0), pat
        assert same(A, Bq), ("decode", pat)
    for local in (False, True):  # a row (global) or a column (local) of the grid
        o.local_or_column = local
        cpl = ecg.CodingParameters(**params, local_or_column=local)
        p.init_coding_parameters(cpl)
        p.set_isvertical(isvertical)
        if local:
            c = rng.randrange(o.k1)
            members = [o.rowcol2bid(r, c) for r in range(o.k2 + o.m2)]
            nd = o.k2
        else:
            r = rng.randrange(o.k2)
            members = [o.rowcol2bid(r, c) for c in range(o.k1 + o.m1)]
            nd = o.k1
        d_all, par = members[:nd], members[nd:]
        sub = rng.sample(d_all, rng.randint(1, nd))
        a, b = E.zeros(len(par), B), E.zeros(len(par), B)
        o.encode_partial_blocks_for_encoding([stripe[i] for i in sub], a, B, sub, par)
        assert p.encode_partial_blocks_for_encoding([stripe[i] for i in sub], b, B, sub, par) == 0
        assert same(a, b), ("partial enc", local, sub, par)
        lost = rng.choice(members)
        surv = [i for i in members if i != lost][:nd]
        lsub = rng.sample(surv, rng.randint(1, nd))
        a, b = E.zeros(1, B), E.zeros(1, B)
        o.encode_partial_blocks_for_decoding([stripe[i] for i in lsub], a, B, lsub, surv, [lost])
        assert p.encode_partial_blocks_for_decoding([stripe[i] for i in lsub], b, B, lsub, surv, [lost]) == 0
        assert same(a, b), ("partial dec", local, lsub, surv, lost)


def test_block_larger_than_2gib(ecg, oracle, torch_cuda):
    """One block of 2^31 + 53 bytes: the jerasure tier's `int size` cannot express it, the batched tier
    takes 64-bit sizes.  Exercises 64-bit offsets in the vector kernel (2^31 + 48 bytes) and the byte
    kernel's tail (5 bytes past it), GENERAL and BINARY, checked against the oracle on windows at the
    start, across the 2 GiB boundary and at the end; the byte after the block stays untouched."""
    torch = torch_cuda
    Bmax = (1 << 31) + 64
    B = (1 << 31) + 53
    st = torch.empty((1, 4, Bmax), dtype=torch.uint8, device="cuda")  # 8 GiB
    ecg.fill_random(st, 77)
    st[0, 2:, B:] = 0xA5
    view = st[:, :, :B]  # strides stay 16-byte multiples; B itself is ragged
    ecg.matrix_apply_batch([[7, 201]], [0, 1], [2], view, view)   # GENERAL
    ecg.matrix_apply_batch([[1, 1]], [0, 1], [3], view, view)     # BINARY
    torch.cuda.synchronize()
    for lo in (0, (1 << 31) - 4096, B - 6000):
        hi = min(B, lo + 8192)
        a, b = st[0, 0, lo:hi].cpu().numpy(), st[0, 1, lo:hi].cpu().numpy()
        ref = [np.zeros(hi - lo, np.uint8)]
        oracle.jerasure_matrix_encode(2, 1, [7, 201], [a, b], ref, hi - lo)
        assert np.array_equal(st[0, 2, lo:hi].cpu().numpy(), ref[0]), lo
        assert np.array_equal(st[0, 3, lo:hi].cpu().numpy(), a ^ b), lo
    assert bool((st[0, 2:, B:] == 0xA5).all())


def test_host_block_at_int_max(ecg, oracle, torch_cuda):
    """The reference's largest expressible block (`int block_size` = 2^31 - 1) through the Jerasure tier
    on host buffers: RS(2,1) encode and a decode of the lost data block, checked against the oracle on
    windows at the start, across 1 GiB, and at the ragged end."""
    torch = torch_cuda
    B = (1 << 31) - 1
    g = torch.empty((2, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(g, 91)
    data = [g[0].cpu().numpy(), g[1].cpu().numpy()]
    del g
    M = ecg.reed_sol_vandermonde_coding_matrix(2, 1)
    coding = [np.zeros(B, np.uint8)]
    ecg.jerasure_matrix_encode(2, 1, M, data, coding, B)
    wins = [(0, 8192), ((1 << 30) - 4096, (1 << 30) + 4096), (B - 8191, B)]
    for lo, hi in wins:
        ref = [np.zeros(hi - lo, np.uint8)]
        oracle.jerasure_matrix_encode(2, 1, M, [data[0][lo:hi], data[1][lo:hi]], ref, hi - lo)
        assert np.array_equal(coding[0][lo:hi], ref[0]), lo
    saved = [data[0][lo:hi].copy() for lo, hi in wins]
    data[0][:] = 0xEE
    assert ecg.jerasure_matrix_decode(2, 1, M, 1, [0, -1], data, coding, B) == 0
    for (lo, hi), want in zip(wins, saved):
        assert np.array_equal(data[0][lo:hi], want), lo


def test_decode_duplicate_erasures(ecg, oracle, torch_cuda):
    """Repeated ids in `erasures` count once (jerasure_erasures_to_erased), so [3, 3] decodes like [3]
    and four distinct losses among repeats are still > m = 3 (-1): host tier and device tier agree with
    the oracle, return codes included."""
    torch = torch_cuda
    k, m, B = 6, 3, 4096 + 9
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    data = [rnd(B, 300 + j) for j in range(k)]
    coding = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data, coding, B)
    for er in ([3, 3], [3, 7, 3, 7], [0, 8, 0, 8, 8], [1, 2, 3, 1, 2, 3, 4]):
        A = [x.copy() for x in data + coding]
        Bh = [x.copy() for x in data + coding]
        for e in er:
            A[e][:] = 0xEE
            Bh[e][:] = 0xEE
        ra = oracle.jerasure_matrix_decode(k, m, M, 1, er + [-1], A[:k], A[k:], B)
        rb = ecg.jerasure_matrix_decode(k, m, M, 1, er + [-1], Bh[:k], Bh[k:], B)
        assert ra == rb and same(A, Bh), er
        dev = [torch.from_numpy(x).cuda() for x in [y.copy() for y in data + coding]]
        for e in er:
            dev[e].fill_(0xEE)
        assert ecg.dev_matrix_decode(k, m, M, 1, er + [-1], dev[:k], dev[k:], B) == ra, er
        torch.cuda.synchronize()
        assert same([x.cpu().numpy() for x in dev], A), er  # undecodable: nothing written, as in the library


@pytest.mark.parametrize("layout", ["strided", "scattered", "unaligned"])
def test_batch_scope_layouts(ecg, oracle, torch_cuda, layout):
    """A batch-scope run whose blocks form one strided batch goes out as a strided launch; scattered
    blocks (random offsets in a pool) as a pointer-table launch; unaligned scattered blocks as a
    pointer-table launch of the byte kernel.  All give the oracle's bytes, for encode and for a decode
    plan of several ops."""
    _batch_scope_layouts(ecg, oracle, torch_cuda, layout)


def _batch_scope_layouts(ecg, oracle, torch, layout):
    k, m, S, B = 6, 3, 24, 8192 + 16
    n = k + m
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    pool = torch.empty(((S * n + 7) * B + 16,), dtype=torch.uint8, device="cuda")
    if layout == "strided":
        offs = [[(s * n + b) * B for b in range(n)] for s in range(S)]
    else:
        slots = list(range(S * n + 7))
        random.Random(4).shuffle(slots)
        offs = [[slots[s * n + b] * B + (3 if layout == "unaligned" else 0) for b in range(n)] for s in range(S)]
    host = [[rnd(B, 1000 + s * n + b) for b in range(k)] for s in range(S)]
    blk = [[pool[o:o + B] for o in offs[s]] for s in range(S)]
    for s in range(S):
        for b in range(k):
            blk[s][b].copy_(torch.from_numpy(host[s][b]))
        for b in range(k, n):
            blk[s][b].fill_(0x5A)
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))
    with ecg.batch():
        for s in range(S):
            ec.encode(blk[s][:k], blk[s][k:], B)
    torch.cuda.synchronize()
    want = []
    for s in range(S):
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, host[s], ref, B)
        want.append(host[s] + ref)
        assert same([x.cpu().numpy() for x in blk[s]], want[s]), (layout, "encode", s)
    for s in range(S):  # lose data 1 and parity 0 everywhere: one decode plan of several ops per call
        blk[s][1].fill_(0xEE)
        blk[s][k].fill_(0xEE)
    with ecg.batch():
        for s in range(S):
            ec.decode(blk[s][:k], blk[s][k:], B, [1, k, -1], 2)
    torch.cuda.synchronize()
    for s in range(S):
        assert same([x.cpu().numpy() for x in blk[s]], want[s]), (layout, "decode", s)


@pytest.mark.parametrize("form", [0, 1, 2])
def test_replay_reference_repair_sequence(ecg, oracle, torch_cuda, form):
    """bench.py's C++ caller of config 3's per-stripe sequence (loopback/replay.cpp): helper partial, main
    partial and perform_addition per stripe through the C ABI -- one launch each (form 0), in scopes
    (1) and in scopes with scratch partials (2) -- rebuilds every lost block (local repairs of every
    data / local-parity block, Azure-LRC(12,2,2)), and the partials are never written in form 2."""
    import sys
    sys.argv = sys.argv[:1]
    import bench
    torch = torch_cuda
    k, l, g, B, S = 12, 2, 2, 4096 + 16, 70
    n = k + g + l
    cp = ecg.CodingParameters(k=k, l=l, g=g, local_or_column=True)
    ec = ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    M = ec.make_encoding_matrix()
    st = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 0x9E7 + form)
    ecg.encode_batch(k, g + l, M, st[:, :k], st[:, k:])
    cls_local = [e for e in range(n) if e not in (12, 13)]
    splits = [bench.azure_local_split(e) for e in cls_local]
    fail = torch.tensor(cls_local, dtype=torch.int32)
    surv = torch.tensor([x[0] for x in splits], dtype=torch.int32).contiguous()
    helper = torch.tensor([x[1][0] for x in splits], dtype=torch.int32).contiguous()
    main = torch.tensor([x[1][1] for x in splits], dtype=torch.int32).contiguous()
    stripe_of = torch.arange(S, dtype=torch.int32)
    pattern_of = (torch.arange(S, dtype=torch.int32) % len(cls_local)).contiguous()
    partials = torch.full((S, 2, B), 0x5A, dtype=torch.uint8, device="cuda")
    out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
    rp = bench.replay_lib()
    rc = rp.ecg_replay_partial_repair(ec._h, form, 16, st.data_ptr(), st.stride(0), st.stride(1), B, S,
                                      stripe_of.data_ptr(), pattern_of.data_ptr(), fail.data_ptr(), 6, surv.data_ptr(),
                                      3, helper.data_ptr(), 3, main.data_ptr(), partials.data_ptr(), out.data_ptr(),
                                      out.stride(0), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, ecg.lib().ecg_last_error()
    torch.cuda.synchronize()
    idx = torch.arange(S, device="cuda")
    lost = torch.tensor(cls_local, device="cuda")[pattern_of.cuda().long()]
    assert torch.equal(out, st[idx, lost])
    if form == 2:
        assert bool((partials == 0x5A).all()), "scratch partials were written"
        assert ecg.batch_last_stats()["composed"] == S - 64  # the last scope: 6 stripes, 3 calls -> 1 each
    else:
        assert not bool((partials == 0x5A).all())
    # one repair against the oracle's own partial decoding (erasure_code.cpp:113-150)
    from oracle import ec_ref as E
    o = E.ec_factory(E.ECTYPE.AZURE_LRC, E.CodingParameters(k=k, l=l, g=g, local_or_column=True))
    o.init_coding_parameters(E.CodingParameters(k=k, l=l, g=g, local_or_column=True))
    host = st[3].cpu().numpy()
    e, (sv, (hs, ms)) = cls_local[3], splits[3]
    p0, p1 = E.zeros(1, B), E.zeros(1, B)
    o.encode_partial_blocks_for_decoding([host[b] for b in hs], p0, B, hs, sv, [e])
    o.encode_partial_blocks_for_decoding([host[b] for b in ms], p1, B, ms, sv, [e])
    assert np.array_equal(p0[0] ^ p1[0], out[3].cpu().numpy())


@pytest.mark.parametrize("form", [0, 1, 2])
def test_replay_reference_merge_sequence(ecg, oracle, torch_cuda, form):
    """bench.py's C++ caller of config 4's per-row sequence (loopback/replay.cpp ecg_replay_merge): per merged
    row, the helper's partial through a PC(8,1,4,1) handle with block ids, the main partial through an
    RS(8,1) handle with columns, and perform_addition -- one launch each (form 0), in scopes (1) and in scopes
    with scratch partials (2) -- gives every row parity of every merge (XOR of the row's 8 blocks of the two
    old PC(4,1,4,1) stripes), and the partials are never written in form 2."""
    import sys
    sys.argv = sys.argv[:1]
    import bench
    torch = torch_cuda
    S, B, nb = 37, 4096 + 16, 25
    blocks = torch.empty((S, 2 * nb, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(blocks, 0x3E6 + form)
    main_ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=8, m=1))
    main_ec.init_coding_parameters(ecg.CodingParameters(k=8, m=1))
    cp = ecg.CodingParameters(k1=8, m1=1, k2=4, m2=1)
    help_ec = ecg.ec_factory(ecg.ECTYPE.PC, cp)
    help_ec.init_coding_parameters(cp)
    plan = bench.pc_merge_plan(nb)
    partials = torch.full((S, 5, 2, B), 0x5A, dtype=torch.uint8, device="cuda")
    out = torch.zeros((S, 5, B), dtype=torch.uint8, device="cuda")
    p = [x.ctypes.data for x in plan]
    rc = bench.replay_lib().ecg_replay_merge(
        main_ec._h, help_ec._h, form, 16, blocks.data_ptr(), blocks.stride(0), blocks.stride(1), B, S, 5, 4,
        p[0], p[1], p[2], 4, p[3], p[4], p[5], partials.data_ptr(), out.data_ptr(), out.stride(0), out.stride(1),
        torch.cuda.current_stream().cuda_stream)
    assert rc == 0, ecg.lib().ecg_last_error()
    torch.cuda.synchronize()
    host = blocks.cpu().numpy()
    mb, hb = plan[0], plan[3]
    for row in range(5):
        want = np.bitwise_xor.reduce(host[:, list(mb[row]) + list(hb[row])], axis=1)
        assert np.array_equal(out[:, row].cpu().numpy(), want), row
    if form == 2:
        assert bool((partials == 0x5A).all()), "scratch partials were written"
        st = ecg.batch_last_stats()  # the last scope: 5 merges, 5 rows, 3 calls -> 1 each
        assert st["recorded"] == 75 and st["composed"] == 25 and st["materialised"] == 0, st
    else:
        assert not bool((partials == 0x5A).all())
