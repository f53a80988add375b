"""The resident call worker (ECG_OPT_CALL_WORKER) against the oracle.

With the option on, small synchronous host-tier calls -- the reference's one jerasure call per stripe on
host buffers (proxy.cpp:312-349), config 1's shape -- are taken by a resident kernel that polls a
descriptor ring instead of one kernel launch per call.  Every byte must be what the launch path and the
oracle give: every input-count bucket, 1-4 outputs, GENERAL and BINARY, block sizes from 4 bytes to
16 KiB (one to sixteen workgroups), decodes, fresh data on every call (stale reads), idle exits and
relaunches, concurrent callers (the ones that find the worker busy take the launch path), and other
streams are not held behind it.  The calls counter proves the worker, not the launch path, ran them."""
import random
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    return torch


ZEROCOPY_DEFAULT = 8 << 20  # the worker takes calls of the zero-copy host path only


@pytest.fixture()
def worker(ecg, torch_cuda):
    saved = ecg.get_option(ecg.ECG_OPT_CALL_WORKER)
    saved_zc = ecg.get_option(ecg.ECG_OPT_ZEROCOPY_BYTES)
    ecg.set_option(ecg.ECG_OPT_CALL_WORKER, 2000)  # exit after 2 ms without a call
    ecg.set_option(ecg.ECG_OPT_ZEROCOPY_BYTES, ZEROCOPY_DEFAULT)  # whatever ECG_ZEROCOPY_BYTES says
    try:
        yield ecg
    finally:
        ecg.set_option(ecg.ECG_OPT_CALL_WORKER, saved)
        ecg.set_option(ecg.ECG_OPT_ZEROCOPY_BYTES, saved_zc)


def rnd(rng, *shape):
    return rng.integers(0, 256, shape, dtype=np.uint8)


def test_worker_shapes_against_oracle(worker, oracle):
    ecg = worker
    rng = np.random.default_rng(5)
    r = random.Random(5)
    before = ecg.call_worker_stats()["calls"]
    n = 0
    for B in (4, 64, 1024, 1028, 4096, 5000, 16384):
        for k in range(1, 17):
            m = r.randint(1, 4)
            kind = r.randrange(3)
            if kind == 0:
                M = [r.randrange(256) for _ in range(k * m)]
            elif kind == 1:
                M = [r.randrange(2) for _ in range(k * m)]  # BINARY flavour
            else:
                M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
            data = list(rnd(rng, k, B))
            want = [np.full(B, 0xA5, np.uint8) for _ in range(m)]  # an all-zero row leaves its output as it was
            got = [x.copy() for x in want]
            oracle.jerasure_matrix_encode(k, m, M, data, want, B)
            for _ in range(2):  # the first call of a new program takes the launch path (tables uploading)
                ecg.jerasure_matrix_encode(k, m, M, data, got, B)
                n += 1
            assert all(np.array_equal(a, b) for a, b in zip(want, got)), (B, k, m, kind)
    st = ecg.call_worker_stats()
    assert not st["disabled"]
    assert st["calls"] - before >= n // 2, st  # at least the second call of every shape ran on the worker


def test_worker_decode_all_single_and_double_erasures(worker, oracle):
    ecg = worker
    k, m, B = 6, 4, 1024
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(9)
    data = list(rnd(rng, k, B))
    coding = [np.zeros(B, np.uint8) for _ in range(m)]
    oracle.jerasure_matrix_encode(k, m, M, data, coding, B)
    before = ecg.call_worker_stats()["calls"]
    pats = [[e] for e in range(k + m)] + [[a, b] for a in range(k + m) for b in range(a + 1, k + m)]
    for rep in range(2):
        for pat in pats:
            d = [x.copy() for x in data]
            c = [x.copy() for x in coding]
            for e in pat:
                (d[e] if e < k else c[e - k])[:] = 0x3C
            assert ecg.jerasure_matrix_decode(k, m, M, 1, pat + [-1], d, c, B) == 0
            assert all(np.array_equal(x, y) for x, y in zip(d + c, data + coding)), pat
    assert ecg.call_worker_stats()["calls"] - before >= len(pats)


def test_worker_never_reads_stale(worker, oracle):
    """Fresh data every call, each output compared before the next call (the flag must follow the bytes)."""
    ecg = worker
    before = ecg.call_worker_stats()["calls"]
    total = 0
    for k, m, B, n in ((6, 4, 1024, 3000), (10, 4, 4096, 800), (10, 4, 16384, 300)):
        M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
        rng = np.random.default_rng(k + B)
        out = [np.zeros(B, np.uint8) for _ in range(m)]
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        bad = 0
        for _ in range(n):
            data = list(rnd(rng, k, B))
            ecg.jerasure_matrix_encode(k, m, M, data, out, B)
            oracle.jerasure_matrix_encode(k, m, M, data, ref, B)
            bad += not all(np.array_equal(a, b) for a, b in zip(out, ref))
        total += n
        assert bad == 0, (k, m, B, bad)
    assert ecg.call_worker_stats()["calls"] - before >= total - 10


def test_worker_exits_when_idle_and_comes_back(worker, oracle):
    """With a 100 us idle limit and 1 ms between calls, every call finds the worker gone: it starts a new
    generation, and the bytes stay right."""
    ecg = worker
    ecg.set_option(ecg.ECG_OPT_CALL_WORKER, 100)
    k, m, B = 6, 4, 1024
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(3)
    ecg.jerasure_matrix_encode(k, m, M, list(rnd(rng, k, B)), [np.zeros(B, np.uint8) for _ in range(m)], B)
    st0 = ecg.call_worker_stats()
    for _ in range(40):
        time.sleep(0.001)
        data = list(rnd(rng, k, B))
        out = [np.zeros(B, np.uint8) for _ in range(m)]
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        ecg.jerasure_matrix_encode(k, m, M, data, out, B)
        oracle.jerasure_matrix_encode(k, m, M, data, ref, B)
        assert all(np.array_equal(a, b) for a, b in zip(out, ref))
    st1 = ecg.call_worker_stats()
    assert st1["calls"] - st0["calls"] == 40 and st1["launches"] - st0["launches"] >= 30, (st0, st1)
    assert not st1["disabled"]


def test_worker_concurrent_callers(worker, oracle):
    """8 threads of calls: one at a time rides the worker, the others take the launch path; all exact."""
    ecg = worker
    k, m, B = 6, 4, 1024
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    errors = []
    before = ecg.call_worker_stats()["calls"]

    def run(t):
        rng = np.random.default_rng(100 + t)
        for _ in range(400):
            data = list(rnd(rng, k, B))
            out = [np.zeros(B, np.uint8) for _ in range(m)]
            ref = [np.zeros(B, np.uint8) for _ in range(m)]
            ecg.jerasure_matrix_encode(k, m, M, data, out, B)
            oracle.jerasure_matrix_encode(k, m, M, data, ref, B)
            if not all(np.array_equal(a, b) for a, b in zip(out, ref)):
                errors.append(t)

    th = [threading.Thread(target=run, args=(t,)) for t in range(8)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors
    assert ecg.call_worker_stats()["calls"] > before


def test_worker_falls_back_outside_its_shapes(worker, oracle):
    """More than 4 outputs, more than 16 inputs, blocks above 16 KiB or not a multiple of 4 bytes: the
    launch path, same bytes."""
    ecg = worker
    rng = np.random.default_rng(21)
    for k, m, B in ((6, 5, 1024), (20, 4, 1024), (6, 4, 32768), (6, 4, 1026)):
        M = [int(x) for x in rnd(rng, k * m)]
        data = list(rnd(rng, k, B))
        want = [np.zeros(B, np.uint8) for _ in range(m)]
        got = [np.zeros(B, np.uint8) for _ in range(m)]
        oracle.jerasure_matrix_encode(k, m, M, data, want, B)
        before = ecg.call_worker_stats()["calls"]
        ecg.jerasure_matrix_encode(k, m, M, data, got, B)
        ecg.jerasure_matrix_encode(k, m, M, data, got, B)
        assert ecg.call_worker_stats()["calls"] == before, (k, m, B)
        assert all(np.array_equal(a, b) for a, b in zip(want, got)), (k, m, B)


def test_worker_does_not_hold_other_streams(worker, oracle, torch_cuda):
    """With the worker resident (long idle limit), work on 8 fresh normal streams completes at once: the
    worker's high-priority stream has its own hardware queue (on a normal stream one of them waited for
    the worker to exit, profiles/r03/persist/queue_interference.log)."""
    torch = torch_cuda
    ecg = worker
    ecg.set_option(ecg.ECG_OPT_CALL_WORKER, 300_000)  # 300 ms idle limit (the worker's own life cap is 50 ms)
    k, m, B = 6, 4, 1024
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(1)
    streams = [torch.cuda.Stream() for _ in range(8)]
    x = torch.zeros(1024, device="cuda")
    for s in streams:  # warm up
        with torch.cuda.stream(s):
            x.add_(1)
        s.synchronize()
    data = list(rnd(rng, k, B))
    out = [np.zeros(B, np.uint8) for _ in range(m)]
    for _ in range(3):
        ecg.jerasure_matrix_encode(k, m, M, data, out, B)  # worker resident now
    worst = 0.0
    for s in streams:
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            x.add_(1)
        s.synchronize()
        worst = max(worst, time.perf_counter() - t0)
    assert worst < 0.010, f"a stream waited {worst * 1e3:.1f} ms behind the worker"


def test_worker_generation_ends_under_load(worker, oracle):
    """Busy or not, a generation takes no call after its 50 ms lifetime: under a continuous stream of calls
    the leader leaves, the waiting call starts the next generation, and no call is lost or wrong."""
    ecg = worker
    k, m, B = 6, 4, 1024
    M = oracle.reed_sol_vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(77)
    ecg.jerasure_matrix_encode(k, m, M, list(rnd(rng, k, B)), [np.zeros(B, np.uint8) for _ in range(m)], B)
    st0 = ecg.call_worker_stats()
    t0 = time.perf_counter()
    n = bad = 0
    while time.perf_counter() - t0 < 0.18:
        data = list(rnd(rng, k, B))
        out = [np.zeros(B, np.uint8) for _ in range(m)]
        ref = [np.zeros(B, np.uint8) for _ in range(m)]
        ecg.jerasure_matrix_encode(k, m, M, data, out, B)
        oracle.jerasure_matrix_encode(k, m, M, data, ref, B)
        bad += not all(np.array_equal(a, b) for a, b in zip(out, ref))
        n += 1
    st1 = ecg.call_worker_stats()
    assert bad == 0
    assert st1["calls"] - st0["calls"] == n
    # 180 ms of calls: at least 3 generations, started by the call that found the last one gone or by one
    # left waiting when it went
    assert st1["launches"] - st0["launches"] >= 3, (st0, st1)
    assert not st1["disabled"]


def test_process_exits_promptly_with_a_resident_worker():
    """A process that exits right after its calls, with the worker resident (idle limit 1 s), exits
    promptly and cleanly: the reaper raises the stop word at exit and the worker leaves at its next poll
    (its 50 ms lifetime would end it soon after anyway); no kernel is left running behind the process."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys, time, numpy as np; sys.path.insert(0, 'erasure-codes-prototype_amd'); import ecg\n"
        "k, m, B = 6, 4, 1024\n"
        "M = ecg.reed_sol_vandermonde_coding_matrix(k, m)\n"
        "d = [np.full(B, j, np.uint8) for j in range(k)]\n"
        "out = [np.zeros(B, np.uint8) for _ in range(m)]\n"
        "for _ in range(3): ecg.jerasure_matrix_encode(k, m, M, d, out, B)\n"
        "st = ecg.call_worker_stats()\n"
        "assert st['calls'] >= 2, st\n"
        "print('T_EXIT', time.time(), flush=True)\n")
    env = dict(os.environ, ECG_CALL_WORKER="1000000", ECG_ZEROCOPY_BYTES=str(ZEROCOPY_DEFAULT))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env, cwd=root)
    t_end = time.time()
    assert p.returncode == 0, p.stderr[-2000:]
    t_exit = float([ln for ln in p.stdout.splitlines() if ln.startswith("T_EXIT")][0].split()[1])
    assert t_end - t_exit < 5.0, f"process took {t_end - t_exit:.2f} s to exit after its last call"
