"""Deferred host-tier calls in a batch scope (ecg_batch_defer_host; engine.cpp record_host / host_flush).

Config 1's shape is the reference's per-stripe host calls (proxy.cpp:312-349): RS(6,4) on 1 KiB blocks,
one jerasure_matrix_encode per stripe.  Inside `with ecg.batch(host=True)` each call stages its inputs
when it is made and its outputs are written when the scope flushes: one H2D, grouped launches, one D2H.
Every result is compared with the oracle on the same bytes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    return torch


def _rs_stripes(rng, S, k, m, B):
    data = [[rng.integers(0, 256, B, dtype=np.uint8) for _ in range(k)] for _ in range(S)]
    coding = [[np.full(B, 0x5A, np.uint8) for _ in range(m)] for _ in range(S)]
    return data, coding


@pytest.mark.parametrize("k,m,B,S", [(6, 4, 1024, 64), (10, 4, 16384, 40), (6, 4, 1000, 17)])
def test_deferred_host_encode_matches_oracle(ecg, oracle, torch_cuda, k, m, B, S):
    rng = np.random.default_rng(k * 1000 + B)
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    data, coding = _rs_stripes(rng, S, k, m, B)
    with ecg.batch(host=True):
        for s in range(S):
            assert ecg.jerasure_matrix_encode(k, m, M, data[s], coding[s], B) == 0
    for s in range(S):
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, data[s], ref, B)
        assert all(np.array_equal(a, b) for a, b in zip(coding[s], ref)), s


def test_deferred_host_inputs_read_at_call_time_and_outputs_at_flush(ecg, oracle, torch_cuda):
    """An input buffer reused right after its call (the proxy's per-stripe staging) does not change that
    call's result; an explicit flush writes the outputs; a second batch then runs on the same scope."""
    k, m, B = 6, 4, 1024
    rng = np.random.default_rng(3)
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    buf = [np.zeros(B, np.uint8) for _ in range(k)]  # one staging set, refilled per stripe
    expect, outs = [], []
    with ecg.batch(host=True) as b:
        for s in range(8):
            for j in range(k):
                buf[j][:] = rng.integers(0, 256, B, dtype=np.uint8)
            ref = [np.zeros(B, np.uint8) for _ in range(m)]
            oracle.jerasure_matrix_encode(k, m, M, buf, ref, B)
            expect.append(ref)
            out = [np.zeros(B, np.uint8) for _ in range(m)]
            assert ecg.jerasure_matrix_encode(k, m, M, buf, out, B) == 0
            outs.append(out)
            if s == 3:
                b.flush()
                assert all(np.array_equal(a, r) for o, e in zip(outs, expect) for a, r in zip(o, e))
    assert all(np.array_equal(a, r) for o, e in zip(outs, expect) for a, r in zip(o, e))


def test_deferred_host_decode_patterns_and_dependences(ecg, oracle, torch_cuda):
    """Per-stripe decodes with different erasure patterns (different plans, erased blocks written in
    place), a decode that reads an encode's pending outputs (the scope flushes first), and a Jerasure
    dotprod, all in one scope."""
    k, m, B, S = 6, 4, 2048, 24
    rng = np.random.default_rng(9)
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    data, coding = _rs_stripes(rng, S, k, m, B)
    with ecg.batch(host=True):
        for s in range(S):
            assert ecg.jerasure_matrix_encode(k, m, M, data[s], coding[s], B) == 0
    for s in range(S):
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, data[s], ref, B)
        assert all(np.array_equal(a, b) for a, b in zip(coding[s], ref)), s
    originals = [[x.copy() for x in data[s]] + [x.copy() for x in coding[s]] for s in range(S)]
    pats = []
    with ecg.batch(host=True):
        for s in range(S):
            e = sorted(rng.choice(k + m, size=1 + s % m, replace=False).tolist())
            pats.append(e)
            for i in e:
                (data[s] + coding[s])[i][:] = 0xEE
            assert ecg.jerasure_matrix_decode(k, m, M, 1, e + [-1], data[s], coding[s], B) == 0
        # a dependent call in the same scope: re-encode stripe 0 from its (pending) decoded data
        c0 = [np.zeros(B, np.uint8) for _ in range(m)]
        assert ecg.jerasure_matrix_encode(k, m, M, data[0], c0, B) == 0
    for s in range(S):
        got = data[s] + coding[s]
        assert all(np.array_equal(a, b) for a, b in zip(got, originals[s])), (s, pats[s])
    assert all(np.array_equal(a, b) for a, b in zip(c0, originals[0][k:]))


@pytest.mark.parametrize("ec_type,params", [(0, dict(k=10, m=4)), (2, dict(k=12, l=2, g=2)),
                                            (7, dict(k1=4, m1=1, k2=4, m2=1))])
def test_deferred_host_facade_calls(ecg, oracle, torch_cuda, ec_type, params):
    """ErasureCode handles in host mode (RS, Azure LRC, PC: multi-op plans) inside a deferred scope:
    encode, then one-block decode per stripe, against the oracle's classes."""
    from oracle import ec_ref as E
    o = E.ec_factory(ec_type, E.CodingParameters(**params))
    p = ecg.ec_factory(ec_type, ecg.CodingParameters(**params))
    k, m, B, S = o.k, o.m, 4096, 12
    rng = np.random.default_rng(ec_type + 5)
    stripes = [[rng.integers(0, 256, B, dtype=np.uint8) for _ in range(k)] for _ in range(S)]
    par = [[np.zeros(B, np.uint8) for _ in range(m)] for _ in range(S)]
    with ecg.batch(host=True):
        for s in range(S):
            assert p.encode(stripes[s], par[s], B) == 0
    for s in range(S):
        ref = E.zeros(m, B)
        o.encode(stripes[s], ref, B)
        assert all(np.array_equal(a, b) for a, b in zip(par[s], ref)), s
    full = [stripes[s] + par[s] for s in range(S)]
    work = [[x.copy() for x in f] for f in full]
    refw = [[x.copy() for x in f] for f in full]
    with ecg.batch(host=True):
        for s in range(S):
            e = s % (k + m)
            work[s][e][:] = 0
            refw[s][e][:] = 0
            rb = p.decode(work[s][:k], work[s][k:], B, [e, -1], 1)
            ra = o.decode(refw[s][:k], refw[s][k:], B, [e, -1], 1)
            assert (ra == 0) == (rb == 0)
    for s in range(S):
        assert all(np.array_equal(a, b) for a, b in zip(work[s], refw[s])), s


def test_deferred_host_mixed_with_device_calls_and_large_blocks(ecg, oracle, torch_cuda):
    """Host calls with blocks above 256 KiB run synchronously inside the scope; a device-tier call flushes
    the pending host calls first; results of every tier equal the oracle's."""
    torch = torch_cuda
    k, m = 4, 2
    rng = np.random.default_rng(21)
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    small = [rng.integers(0, 256, 1024, dtype=np.uint8) for _ in range(k)]
    big = [rng.integers(0, 256, 300 * 1024, dtype=np.uint8) for _ in range(k)]
    cs = [np.zeros(1024, np.uint8) for _ in range(m)]
    cb = [np.zeros(300 * 1024, np.uint8) for _ in range(m)]
    d = torch.from_numpy(np.stack(small + [np.zeros(1024, np.uint8)] * m)).cuda()
    with ecg.batch(host=True):
        assert ecg.jerasure_matrix_encode(k, m, M, small, cs, 1024) == 0   # deferred
        assert ecg.jerasure_matrix_encode(k, m, M, big, cb, 300 * 1024) == 0  # synchronous
        assert all(np.array_equal(a, b) for a, b in zip(cs, cs))  # (pending or done: not inspected)
        ecg.dev_matrix_encode(k, m, M, [d[j] for j in range(k)], [d[k + i] for i in range(m)], 1024)
    torch.cuda.synchronize()
    for blocks, out, B in ((small, cs, 1024), (big, cb, 300 * 1024)):
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, blocks, ref, B)
        assert all(np.array_equal(a, b) for a, b in zip(out, ref)), B
    ref = [np.zeros(1024, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, small, ref, 1024)
    assert np.array_equal(d[k:].cpu().numpy(), np.stack(ref))


def test_defer_host_outside_scope_refused(ecg, torch_cuda):
    assert ecg.lib().ecg_batch_defer_host(1) != 0


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_deferred_host_random_sequences_match_sequential(ecg, oracle, torch_cuda, seed):
    """Random host-tier call sequences over a small pool of shared buffers, so that calls read blocks an
    earlier call of the scope writes (the scope must flush first), overwrite blocks an earlier call read
    (its inputs were staged at call time), write a block twice, change block size mid-scope, flush
    explicitly, and run dotprods and region XORs between encodes.  The GF arithmetic of every call is the
    oracle's (jerasure_matrix_encode / dotprod restated).  The pool after the scope must equal the
    oracle applying the same calls one by one."""
    rng = np.random.default_rng(seed)
    sizes = (1024, 4112) if seed % 2 else (64, 2048)
    pools = {B: [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(12)] for B in sizes}
    ref = {B: [x.copy() for x in pool] for B, pool in pools.items()}
    with ecg.batch(host=True) as b:
        for i in range(160):
            B = sizes[int(rng.integers(0, 4)) == 0]  # mostly the first size: block-size changes flush
            pool, rp = pools[B], ref[B]
            kind = int(rng.integers(0, 10))
            if kind < 7:  # encode: k data blocks -> m coding blocks, all distinct
                k, m = int(rng.integers(1, 7)), int(rng.integers(1, 4))
                ids = rng.choice(len(pool), size=k + m, replace=False).tolist()
                M = [int(x) for x in rng.integers(0, 256, k * m)]
                assert ecg.jerasure_matrix_encode(k, m, M, [pool[j] for j in ids[:k]],
                                                  [pool[j] for j in ids[k:]], B) == 0
                oracle.jerasure_matrix_encode(k, m, M, [rp[j] for j in ids[:k]], [rp[j] for j in ids[k:]], B)
            elif kind < 9:  # dotprod into one block
                k = int(rng.integers(1, 6))
                ids = rng.choice(len(pool), size=k + 1, replace=False).tolist()
                row = [int(x) for x in rng.integers(1, 256, k)]
                assert ecg.jerasure_matrix_dotprod(k, row, None, k, [pool[j] for j in ids[:k]],
                                                   [pool[ids[k]]], B) == 0
                oracle.jerasure_matrix_dotprod(k, row, None, k, [rp[j] for j in ids[:k]], [rp[ids[k]]], B)
            elif kind < 10 and i % 2:  # region XOR (host regions: flushes the pending calls first)
                src, dst = rng.choice(len(pool), size=2, replace=False).tolist()
                assert ecg.galois_region_xor(pool[src], pool[dst], B) == 0
                rp[dst] ^= rp[src]
            else:
                b.flush()
    for B in sizes:
        for j, (a, r) in enumerate(zip(pools[B], ref[B])):
            assert np.array_equal(a, r), (seed, B, j)


@pytest.mark.parametrize("shift", [1, 16, 500, 1023])
def test_deferred_host_partially_overlapping_blocks(ecg, oracle, torch_cuda, shift):
    """blocks of one scope need not be identical-or-disjoint.  Call 1 writes its parities into a
    caller buffer; call 2 reads a block that starts `shift` bytes into call 1's first parity (an offset view
    of the same buffer).  Call 2 must read call 1's output, not the bytes staged before it: the pending
    outputs are compared by byte range, so call 2 flushes the batch first.  Both against the oracle run
    call by call."""
    k, m, B = 6, 4, 1024
    rng = np.random.default_rng(shift)
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    data1 = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(k)]
    region = rng.integers(0, 256, (m + 1) * B, dtype=np.uint8)  # call 1's parities live in region[0:m*B]
    out1 = [region[i * B:(i + 1) * B] for i in range(m)]
    data2 = [region[shift:shift + B]] + [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(k - 1)]
    out2 = [np.zeros(B, np.uint8) for _ in range(m)]
    # the oracle, call by call on copies of the same buffers
    r_region = region.copy()
    r_out1 = [r_region[i * B:(i + 1) * B] for i in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data1, r_out1, B)
    r_data2 = [r_region[shift:shift + B].copy()] + [d.copy() for d in data2[1:]]
    r_out2 = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, r_data2, r_out2, B)
    with ecg.batch(host=True):
        assert ecg.jerasure_matrix_encode(k, m, M, data1, out1, B) == 0
        assert ecg.jerasure_matrix_encode(k, m, M, data2, out2, B) == 0
    assert np.array_equal(region, r_region)
    assert all(np.array_equal(a, b) for a, b in zip(out2, r_out2))
