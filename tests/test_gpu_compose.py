"""GPU parity of composed product-code calls (codes.cpp finish_plan, matrix.cpp compose_chain).

A product-code encode runs its row codes, then its column codes over the data and the row parities just written
(pc.cpp:39-76); the iterative decode alternates column and row decodes (pc.cpp:79-195, HVPC pc.cpp:921-1029).
The facade plans each call as such a chain and runs it composed into ONE region product over the call's inputs.
Every output here is compared, byte for byte, with the oracle's restatement of the reference classes
(oracle/ec_ref.py), and the traffic counters (ecg_traffic_counters) show the composed call: one launch, each
input read once, each output written once.
"""
import itertools
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PC, HPC, HVPC = 7, 8, 9


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    return torch


def same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


def make_pair(ecg, t, params, isvertical=None):
    from oracle import ec_ref as E
    cp = E.CodingParameters(**params)
    o = E.ec_factory(t, cp)
    o.init_coding_parameters(cp)
    p = ecg.ec_factory(t, ecg.CodingParameters(**params))
    p.init_coding_parameters(ecg.CodingParameters(**params))
    if isvertical is not None:
        o.isvertical = isvertical
        p.set_isvertical(isvertical)
    return o, p


def counted(ecg, fn):
    t0 = ecg.traffic_counters()
    r = fn()
    t1 = ecg.traffic_counters()
    return r, t1["launches"] - t0["launches"], t1["bytes"] - t0["bytes"]


# (type, params, isvertical): the BASELINE product-code shape in every class and orientation
SHAPES_4141 = [(PC, {}, None), (HPC, dict(x=2, seri_num=0), True), (HPC, dict(x=2, seri_num=1), False),
               (HVPC, {}, None)]


@pytest.mark.parametrize("t,extra,isv", SHAPES_4141)
@pytest.mark.parametrize("tier", ["host", "device"])
def test_product_code_encode_one_pass(ecg, oracle, torch_cuda, t, extra, isv, tier):
    """(4,1,4,1) encode: bit-exact, ONE launch, every data block read once and every parity written once
    (PC / HPC: 16 in + 9 out = 25 B; HVPC, no global parity: 16 + 8 = 24 B)."""
    torch = torch_cuda
    from oracle import ec_ref as E
    o, p = make_pair(ecg, t, dict(k1=4, m1=1, k2=4, m2=1, **extra), isv)
    B = 65536
    data = E.blocks(o.k, B, 21 + t)
    ca = E.zeros(o.m, B)
    o.encode(data, ca, B)
    if tier == "host":
        cb = E.zeros(o.m, B)
        rc, launches, moved = counted(ecg, lambda: p.encode(data, cb, B))
    else:
        dd = [torch.from_numpy(x).cuda() for x in data]
        dc = [torch.full((B,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(o.m)]
        rc, launches, moved = counted(ecg, lambda: p.encode(dd, dc, B))
        torch.cuda.synchronize()
        cb = [c.cpu().numpy() for c in dc]
    assert rc == 0
    assert same(ca, cb)
    assert launches == 1, launches
    assert moved == (o.k + o.m) * B, (moved // B, o.k + o.m)


def _patterns(n, fmax):
    for f in range(1, fmax + 1):
        yield from itertools.combinations(range(n), f)


@pytest.mark.parametrize("t,extra,isv", SHAPES_4141)
def test_product_code_every_pattern_up_to_3(ecg, oracle, torch_cuda, t, extra, isv):
    """Every erasure pattern of 1-3 blocks of a (4,1,4,1) stripe (2625 patterns; HVPC 2324): the composed
    decode against the oracle's iterative decode, garbage in the erased blocks; same status (decodable or
    not) and the same bytes in every block -- an undecodable pattern still runs the work planned before the
    planner gave up, in both."""
    from oracle import ec_ref as E
    o, p = make_pair(ecg, t, dict(k1=4, m1=1, k2=4, m2=1, **extra), isv)
    B = 1024 + 16
    data = E.blocks(o.k, B, 5 + t)
    coding = E.zeros(o.m, B)
    o.encode(data, coding, B)
    stripe = data + coding
    n = o.k + o.m
    bad, decodable = [], 0
    for pat in _patterns(n, 3):
        A = [x.copy() for x in stripe]
        Bq = [x.copy() for x in stripe]
        for i in pat:
            A[i][:] = 0xE7
            Bq[i][:] = 0xE7
        ra = o.decode(A[:o.k], A[o.k:], B, list(pat) + [-1], len(pat))
        rb = p.decode(Bq[:o.k], Bq[o.k:], B, list(pat) + [-1], len(pat))
        if (ra == 0) != (rb == 0) or not same(A, Bq):
            bad.append(pat)
        if ra == 0:
            decodable += 1
            assert same(A, stripe), pat
    assert not bad, bad[:5]
    assert decodable > n  # every single loss and most double losses


@pytest.mark.parametrize("t,extra,isv", SHAPES_4141)
def test_product_code_decode_composes(ecg, oracle, torch_cuda, t, extra, isv):
    """A pattern the iterative decode chains -- (r0,c0), (r0,c1), (r1,c0): column c1 first, then rows r0
    (reading the block column c1 just rebuilt) and r1 -- runs as one launch that reads no rebuilt block, on
    the device tier, bit-exact."""
    torch = torch_cuda
    from oracle import ec_ref as E
    o, p = make_pair(ecg, t, dict(k1=4, m1=1, k2=4, m2=1, **extra), isv)
    B = 32768
    data = E.blocks(o.k, B, 9)
    coding = E.zeros(o.m, B)
    o.encode(data, coding, B)
    stripe = data + coding
    pat = [o.rowcol2bid(0, 0), o.rowcol2bid(0, 1), o.rowcol2bid(1, 0)]
    A = [x.copy() for x in stripe]
    ra = o.decode(A[:o.k], A[o.k:], B, pat + [-1], len(pat))
    assert ra == 0 and same(A, stripe)
    dev = [torch.from_numpy(x).cuda() for x in stripe]
    for i in pat:
        dev[i].fill_(0xE7)
    rb, launches, moved = counted(ecg, lambda: p.decode(dev[:o.k], dev[o.k:], B, pat + [-1], len(pat)))
    torch.cuda.synchronize()
    assert rb == 0
    assert same([x.cpu().numpy() for x in dev], stripe)
    assert launches == 1, launches
    # chained: 3 ops of 4 -> 1 (16 blocks); composed: the survivors the three values need, read once
    assert moved < 3 * 5 * B, moved // B


@pytest.mark.parametrize("t,params", [(PC, dict(k1=3, m1=2, k2=3, m2=2)), (HVPC, dict(k1=3, m1=2, k2=3, m2=2)),
                                      (HPC, dict(k1=3, m1=2, k2=2, m2=2, x=2, seri_num=1)),
                                      (PC, dict(k1=5, m1=1, k2=2, m2=2))])
def test_general_product_codes_compose(ecg, oracle, torch_cuda, t, params):
    """GENERAL (non-0/1) row and column codes: encode and 150 random patterns of 1-4 losses against the
    oracle, host tier."""
    from oracle import ec_ref as E
    o, p = make_pair(ecg, t, params, True if t == HPC else None)
    B = 4096 + 48
    data = E.blocks(o.k, B, 31)
    ca, cb = E.zeros(o.m, B), E.zeros(o.m, B)
    o.encode(data, ca, B)
    rc, launches, _ = counted(ecg, lambda: p.encode(data, cb, B))
    assert rc == 0 and same(ca, cb)
    assert launches <= 2  # one composed op (a tail launch would be a second kernel; B % 16 == 0 here)
    stripe = data + ca
    n = o.k + o.m
    rng = random.Random(t * 100 + o.k)
    for _ in range(150):
        pat = rng.sample(range(n), rng.randint(1, 4))
        A = [x.copy() for x in stripe]
        Bq = [x.copy() for x in stripe]
        for i in pat:
            A[i][:] = 0x3C
            Bq[i][:] = 0x3C
        ra = o.decode(A[:o.k], A[o.k:], B, pat + [-1], len(pat))
        rb = p.decode(Bq[:o.k], Bq[o.k:], B, pat + [-1], len(pat))
        assert (ra == 0) == (rb == 0), pat
        assert same(A, Bq), pat


def test_product_code_encode_in_batch_scope(ecg, oracle, torch_cuda):
    """The proxy's per-stripe encode loop (proxy.cpp:312-349) on PC(4,1,4,1) device blocks inside a batch
    scope: one strided launch for all stripes, 25 B per stripe, every parity against the oracle."""
    torch = torch_cuda
    from oracle import ec_ref as E
    o, p = make_pair(ecg, PC, dict(k1=4, m1=1, k2=4, m2=1))
    S, B = 64, 16384
    stripes = torch.empty((S, o.k + o.m, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 0xC0DE)

    def run():
        with ecg.batch():
            for s in range(S):
                assert p.encode([stripes[s, j] for j in range(o.k)], [stripes[s, o.k + j] for j in range(o.m)], B) == 0

    _, launches, moved = counted(ecg, run)
    torch.cuda.synchronize()
    assert launches == 1, launches
    assert moved == S * (o.k + o.m) * B
    host = stripes.cpu().numpy()
    for s in (0, 17, S - 1):
        coding = E.zeros(o.m, B)
        o.encode([host[s, j] for j in range(o.k)], coding, B)
        assert same(coding, [host[s, o.k + j] for j in range(o.m)]), s
