"""Drop-in check of the Jerasure-compatible tier through include/jerasure_shim/.

tests/shim/consumer.cpp calls the seven Jerasure symbols hhlgt/erasure-codes-prototype uses (SURVEY.md
§8(a) rows a1-a7) with the reference's argument shapes, through the shim headers only, linked against
libecg.so (built by the package Makefile as bin/jerasure_shim_consumer).  The CPU test checks the
host-side builders (no GPU needed); the GPU test checks every byte it produces against the oracle.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "erasure-codes-prototype_amd")
BIN = os.path.join(PKG, "bin", "jerasure_shim_consumer")


@pytest.fixture(scope="module")
def consumer(ecg):
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", PKG, "bin/jerasure_shim_consumer"])
    return BIN


def _parse(out):
    res = {}
    for line in out.strip().splitlines():
        name, *vals = line.split()
        res[name] = [int(v) for v in vals]
    return res


def test_shim_matrices(consumer, oracle):
    out = subprocess.run([consumer, "matrices"], capture_output=True, text=True, check=True).stdout
    r = _parse(out)
    assert r["rs_10_4"] == oracle.reed_sol_vandermonde_coding_matrix(10, 4)
    assert r["cauchy_good_12_3"] == oracle.cauchy_good_general_coding_matrix(12, 3)
    k = 4
    M = oracle.reed_sol_vandermonde_coding_matrix(k, 2)
    F = [[int(i == j) for j in range(k)] for i in range(k)] + [M[i * k:(i + 1) * k] for i in range(2)]
    S = sum((F[i] for i in (1, 2, 3, 4)), [])
    rc, inv = oracle.jerasure_invert_matrix(S, k)
    assert r["invert_rc"] == [rc] == [0]
    assert r["inverse"] == inv
    assert r["decode_row"] == oracle.jerasure_matrix_multiply(F[0], inv, 1, k, k, k)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B", [(10, 4, 4099), (6, 4, 1024), (12, 3, 65536)])
def test_shim_bytes(consumer, oracle, tmp_path, k, m, B):
    rng = np.random.default_rng(k * 100 + m)
    data = rng.integers(0, 256, (k, B), dtype=np.uint8)
    inp, outp = tmp_path / "in.bin", tmp_path / "out.bin"
    data.tofile(inp)
    p = subprocess.run([consumer, "bytes", str(inp), str(outp), str(k), str(m), str(B)], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "decode_rc 0" in p.stdout and "failed" not in p.stderr, (p.stdout, p.stderr)
    got = np.fromfile(outp, dtype=np.uint8).reshape(m + 4, B)
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    coding = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, list(data), coding, B)
    for i in range(m):
        assert np.array_equal(got[i], coding[i]), f"coding {i}"
    assert np.array_equal(got[m], data[0]), "decoded data 0"
    assert np.array_equal(got[m + 1], coding[1]), "decoded coding 1"
    # partial decoding of block 0 from survivors 1..k, local half 1..k/2 (erasure_code.cpp:113-150)
    F = [[int(i == j) for j in range(k)] for i in range(k)] + [M[i * k:(i + 1) * k] for i in range(m)]
    rc, inv = oracle.jerasure_invert_matrix(sum((F[i] for i in range(1, k + 1)), []), k)
    R = oracle.jerasure_matrix_multiply(F[0], inv, 1, k, k, k)
    nloc = k // 2
    blocks = list(data) + coding
    part = [np.zeros(B, np.uint8)]
    oracle.jerasure_matrix_encode(nloc, 1, R[:nloc], [blocks[i + 1] for i in range(nloc)], part, B)
    assert np.array_equal(got[m + 2], part[0]), "partial"
    assert np.array_equal(got[m + 3], data[0] ^ data[1]), "galois_region_xor"


FACADE = os.path.join(PKG, "bin", "facade_consumer")


@pytest.fixture(scope="module")
def facade_consumer(ecg):
    if not os.path.exists(FACADE):
        subprocess.check_call(["make", "-s", "-C", PKG, "bin/facade_consumer"])
    return FACADE


def test_facade_cpp_plans(facade_consumer):
    """INTEGRATION.md Option B compiles and links: ecg::ec_factory + the C++ classes, no GPU needed for
    matrices and repair planning (Azure-LRC(12,2,2), block 0, OPTIMAL partition)."""
    from oracle import ec_ref as E
    out = subprocess.run([facade_consumer, "plans"], capture_output=True, text=True, check=True).stdout.splitlines()
    M = [int(x) for x in out[0].split()[1:]]
    assert M == E.ec_factory(E.ECTYPE.AZURE_LRC, E.CodingParameters(k=12, l=2, g=2)).make_encoding_matrix()
    plan = out[1].split("|")
    assert plan[0].split() == ["plan", "1"]  # a local plan
    assert [sorted(int(x) for x in h.split()) for h in plan[1:]] == [[1, 2], [3, 4, 5], [14]]


@pytest.mark.gpu
def test_facade_cpp_bytes(facade_consumer, oracle, tmp_path):
    """The same consumer on the GPU: Azure(12,2,2) encode and the partial-decoding repair of block 0
    (helper partial + main partial + perform_addition) byte-for-byte against the oracle."""
    from oracle import ec_ref as E
    B = 65536 + 5
    data = np.random.default_rng(12).integers(0, 256, (12, B), dtype=np.uint8)
    inp, outp = tmp_path / "in.bin", tmp_path / "out.bin"
    data.tofile(inp)
    p = subprocess.run([facade_consumer, "bytes", str(inp), str(outp), str(B)], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    got = np.fromfile(outp, dtype=np.uint8).reshape(5, B)
    ec = E.ec_factory(E.ECTYPE.AZURE_LRC, E.CodingParameters(k=12, l=2, g=2))
    coding = E.zeros(4, B)
    ec.encode(list(data), coding, B)
    for i in range(4):
        assert np.array_equal(got[i], coding[i]), i
    assert np.array_equal(got[4], data[0])
