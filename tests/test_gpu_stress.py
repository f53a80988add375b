"""Concurrency soak of the engine's shared state (GPU): the proxy issues EC calls from detached threads
(proxy.cpp:416-419), so every tier must stay exact when calls from several threads interleave.

Eight threads issue 400 random operations each, at once.  Each operation is one of:
- host-tier encode / decode / partial decode of a random code family, with small (staged, zero-copy)
  and large (pageable-copy) blocks;
- device-tier encode on HBM blocks, sometimes inside a deferred-batch scope.

The coefficient-program cache is shrunk to 8 entries, so programs are evicted while other threads'
launches may still use them.  Every result is compared with the oracle.  This test caught a GPU fault in
an earlier design that registered the caller's pages for large host calls (see engine.cpp run_host).
"""
import os
import random
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FAMILIES = [(0, dict(k=10, m=4)), (0, dict(k=6, m=3)), (1, dict(k=4, m=2, x=2, seri_num=1)),
            (2, dict(k=12, l=2, g=2)), (3, dict(k=8, l=3, g=2)), (4, dict(k=8, l=2, g=2)),
            (5, dict(k=8, l=2, g=2)), (6, dict(k=8, l=2, g=2)), (7, dict(k1=4, m1=1, k2=4, m2=1)),
            (9, dict(k1=4, m1=2, k2=2, m2=1))]


def _worker(tid, ecg, torch, n_ops, errors):
    from oracle import ec_ref as E
    rng = random.Random(1000 + tid)
    try:
        for op in range(n_ops):
            t, params = FAMILIES[rng.randrange(len(FAMILIES))]
            o = E.ec_factory(t, E.CodingParameters(**params))
            p = ecg.ec_factory(t, ecg.CodingParameters(**params))
            k, m = o.k, o.m
            B = rng.choice([64, 1000, 4096, 300 * 1024])  # 300 KiB: the pinned large-block path
            data = [np.random.default_rng(tid * 100000 + op * 16 + j).integers(0, 256, B, dtype=np.uint8)
                    for j in range(k)]
            ref = E.zeros(m, B)
            o.encode(data, ref, B)
            kind = rng.randrange(4)
            if kind == 0:  # host encode
                got = [np.full(B, 0x33, np.uint8) for _ in range(m)]
                assert p.encode(data, got, B) == 0
                assert all(np.array_equal(a, b) for a, b in zip(got, ref)), ("host encode", t, params, B)
            elif kind == 1:  # host decode of one lost block
                stripe = [x.copy() for x in data] + [x.copy() for x in ref]
                e = rng.randrange(k + m)
                stripe[e][:] = 0
                a = [x.copy() for x in stripe]
                ra = o.decode(a[:k], a[k:], B, [e, -1], 1)
                rb = p.decode(stripe[:k], stripe[k:], B, [e, -1], 1)
                assert (ra == 0) == (rb == 0)
                assert all(np.array_equal(x, y) for x, y in zip(a, stripe)), ("host decode", t, params, e)
            elif kind == 2:  # device encode, alone or inside a deferred-batch scope
                d = torch.from_numpy(np.stack(data + ref)).cuda()
                d[k:] = 0
                if rng.random() < 0.5:
                    with ecg.batch():
                        p.encode([d[j] for j in range(k)], [d[k + i] for i in range(m)], B)
                else:
                    p.encode([d[j] for j in range(k)], [d[k + i] for i in range(m)], B)
                torch.cuda.current_stream().synchronize()
                h = d.cpu().numpy()
                assert all(np.array_equal(h[k + i], ref[i]) for i in range(m)), ("device encode", t, params, B)
            else:  # host partial encode over a random data subset == XOR-able share of the parities
                if t >= 7:
                    continue
                npar = o.g if hasattr(o, "g") else m
                par = list(range(k, k + npar))
                sub = sorted(rng.sample(range(k), rng.randint(1, k)))
                a, b = E.zeros(npar, B), E.zeros(npar, B)
                o.encode_partial_blocks_for_encoding([data[i] for i in sub], a, B, sub, par)
                assert p.encode_partial_blocks_for_encoding([data[i] for i in sub], b, B, sub, par) == 0
                assert all(np.array_equal(x, y) for x, y in zip(a, b)), ("partial", t, params, sub)
    except Exception as e:  # noqa: BLE001
        errors.append((tid, repr(e)))


@pytest.mark.parametrize("call_worker", [0, 2000])
def test_concurrent_mixed_tiers_with_cache_eviction(ecg, oracle, call_worker):
    """... also with the resident call worker on (ECG_OPT_CALL_WORKER): it takes one thread's small host
    calls at a time while the programs it reads are being evicted by the others."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("needs an MI355X")
    saved = ecg.get_option(ecg.ECG_OPT_PROGRAM_CACHE)
    saved_worker = ecg.get_option(ecg.ECG_OPT_CALL_WORKER)
    saved_zc = ecg.get_option(ecg.ECG_OPT_ZEROCOPY_BYTES)
    errors = []
    try:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, 8)
        ecg.set_option(ecg.ECG_OPT_CALL_WORKER, call_worker)
        if call_worker:  # the worker takes calls of the zero-copy host path only
            ecg.set_option(ecg.ECG_OPT_ZEROCOPY_BYTES, 8 << 20)
        n_ops = int(os.environ.get("ECG_SOAK_OPS", "400"))  # longer soaks: ECG_SOAK_OPS=2000
        th = [threading.Thread(target=_worker, args=(t, ecg, torch, n_ops, errors)) for t in range(8)]
        [x.start() for x in th]
        [x.join(timeout=100 + n_ops // 10) for x in th]
        assert not any(x.is_alive() for x in th), "a worker hung"
    finally:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, saved)
        ecg.set_option(ecg.ECG_OPT_CALL_WORKER, saved_worker)
        ecg.set_option(ecg.ECG_OPT_ZEROCOPY_BYTES, saved_zc)
    assert not errors, errors[:5]
    if call_worker:
        st = ecg.call_worker_stats()
        assert st["calls"] > 0 and not st["disabled"], st


def test_thread_per_request_resources_bounded(ecg, oracle):
    """The proxy starts a new detached thread per SET (proxy.cpp:416-419) and calls the codec from it.
    Host-tier contexts (stream, device scratch, pinned staging) are leased per call from a pool, so 240
    short-lived threads, at most 6 alive at once, create at most 6 new contexts; pointer-table slots are
    per device, not per thread.  Every result is checked against the oracle."""
    import torch
    from oracle import ec_ref as E
    before = ecg.lib().ecg_host_contexts()
    errors = []
    o = E.ec_factory(0, E.CodingParameters(k=6, m=3))

    def one(i):
        try:
            p = ecg.ec_factory(0, ecg.CodingParameters(k=6, m=3))
            B = 4096 if i % 3 else 300 * 1024
            data = [np.random.default_rng(i * 10 + j).integers(0, 256, B, dtype=np.uint8) for j in range(6)]
            ref = E.zeros(3, B)
            o.encode(data, ref, B)
            got = [np.zeros(B, np.uint8) for _ in range(3)]
            assert p.encode(data, got, B) == 0
            assert all(np.array_equal(a, b) for a, b in zip(got, ref)), ("host", i)
            if i % 4 == 0:  # pointer-table launch (region_xor_batch) from this short-lived thread
                a = torch.from_numpy(np.stack(data[:2])).cuda()
                b = torch.from_numpy(np.stack(data[2:4])).cuda()
                ecg.region_xor_batch(a, b)
                torch.cuda.current_stream().synchronize()
                assert np.array_equal(b.cpu().numpy(), np.stack(data[:2]) ^ np.stack(data[2:4])), ("xor", i)
        except Exception as e:  # noqa: BLE001
            errors.append((i, repr(e)))

    for wave in range(40):
        th = [threading.Thread(target=one, args=(wave * 6 + t,)) for t in range(6)]
        [x.start() for x in th]
        [x.join(timeout=60) for x in th]
        assert not any(x.is_alive() for x in th), "a worker hung"
    assert not errors, errors[:5]
    assert ecg.lib().ecg_host_contexts() - before <= 6


def test_eviction_does_not_stall_other_streams(ecg, oracle):
    """Program-cache eviction retires the evicted tables with a cover event recorded on each stream they ran
    on the next time a caller hands the library that stream (engine.hpp ProgramSet); it neither
    synchronizes the device nor frees device memory (hipFree would).  A second stream keeps
    ~0.4 s of encodes queued while this thread makes 24 calls that each evict: they must take no longer
    than the same 24 launches with their programs already cached (the control; streams can share one of
    the runtime's hardware queues, GPU_MAX_HW_QUEUES = 4, and then both wait alike), and every evicted set
    is freed once its launches completed."""
    import time

    import torch
    saved = ecg.get_option(ecg.ECG_OPT_PROGRAM_CACHE)
    try:
        k, m, S, B = 10, 4, 256, 1 << 20
        M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
        big = torch.empty((S, k + m, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(big, 0xE71C)
        rng = np.random.default_rng(7)
        mine = torch.cuda.Stream()
        Bs = 4096
        blocks = torch.from_numpy(rng.integers(0, 256, (6, Bs), dtype=np.uint8)).cuda()
        mats = [[int(x) for x in rng.integers(1, 256, 4 * 2)] for _ in range(24)]
        outs = [torch.zeros((2, Bs), dtype=torch.uint8, device="cuda") for _ in mats]
        busy = torch.cuda.Stream()
        # everything the calls use is ready before a busy queue exists: a synchronize of the default
        # stream after it would wait for the busy stream too (legacy default-stream semantics)
        torch.cuda.synchronize()
        ecg.encode_batch(k, m, M, big[:, :k], big[:, k:], stream=busy.cuda_stream)  # program built up front
        busy.synchronize()
        t0 = time.time()
        ecg.encode_batch(k, m, M, big[:, :k], big[:, k:], stream=busy.cuda_stream)
        busy.synchronize()
        one = time.time() - t0
        reps = max(20, int(0.4 / max(one, 1e-4)))  # ~0.4 s queued on `busy`

        def timed_calls():
            for _ in range(reps):
                ecg.encode_batch(k, m, M, big[:, :k], big[:, k:], stream=busy.cuda_stream)
            t0 = time.time()
            for Mi, out in zip(mats, outs):
                ecg.dev_matrix_encode(4, 2, Mi, [blocks[j] for j in range(4)], [out[0], out[1]], Bs,
                                      stream=mine.cuda_stream)
            mine.synchronize()
            dt = time.time() - t0
            busy.synchronize()
            return dt

        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, 4096)
        assert ecg.lib().ecg_program_sets_reclaim() == 0  # earlier tests' sets whose streams are gone
        timed_calls()  # programs built and cached
        control = timed_calls()  # the same launches, no eviction
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, 2)
        evicting = timed_calls()  # every call builds its program again and evicts
        # A device-wide synchronize on the eviction path would make the evicting calls wait for the whole
        # queue (~0.4 s); scheduling noise on a shared GPU is far below that.  So the bound is a quarter of
        # the queued time, not a fixed few ms; the timings are printed as the metric.
        queued = reps * one
        print(f"eviction: {evicting * 1e3:.1f} ms vs control {control * 1e3:.1f} ms, {queued * 1e3:.0f} ms queued")
        assert evicting < control + max(0.05, 0.25 * queued), (
            f"evicting calls {evicting:.3f} s vs control {control:.3f} s ({reps} x {one * 1e3:.2f} ms queued "
            f"on the other stream)")
        host = blocks.cpu().numpy()
        for Mi, out in zip(mats, outs):
            want = [np.zeros(Bs, np.uint8) for _ in range(2)]
            oracle.jerasure_matrix_encode(4, 2, Mi, [host[j] for j in range(4)], want, Bs)
            assert np.array_equal(out.cpu().numpy(), np.stack(want))
        torch.cuda.synchronize()
        # sets used on `mine` were covered by later calls on it; the encode's set, evicted by `mine`'s calls,
        # waits for `busy` to be handed over again -- one more call on it frees it without any synchronize
        ecg.encode_batch(k, m, M, big[:, :k], big[:, k:], stream=busy.cuda_stream)
        ecg.dev_matrix_encode(4, 2, mats[0], [blocks[j] for j in range(4)], [outs[0][0], outs[0][1]], Bs,
                              stream=mine.cuda_stream)
        torch.cuda.synchronize()
        left = ecg.lib().ecg_program_sets_retiring()
        assert left <= 2, left  # at most the sets of the last two calls, still current
        assert ecg.lib().ecg_program_sets_reclaim() == 0
    finally:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, saved)


def _hip():
    """The HIP runtime torch loaded (same soname as libecg's), for raw caller streams."""
    import ctypes
    h = ctypes.CDLL("libamdhip64.so.7")
    h.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    h.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    h.hipStreamQuery.argtypes = [ctypes.c_void_p]
    return h


def test_eviction_retires_across_destroyed_and_reused_streams(ecg, oracle):
    """The reference runs each EC call on a detached thread (proxy.cpp:416-419); an integrator with a stream
    per request creates and DESTROYS raw HIP streams.  The runtime hands a destroyed handle to the next
    hipStreamCreate, so a stored handle may name a dead stream or an unrelated new one.  Program sets used
    on such streams are evicted (cache of 2) by calls on other streams; nothing the library keeps may name
    a caller stream after the call returns, and every result is checked against the oracle.  Round 3
    crashed here (gpurun_out/evict.log)."""
    import ctypes

    import torch
    bt = os.path.join(os.path.dirname(os.path.abspath(__file__)), "segv", "libsegv_bt.so")
    if os.path.exists(bt):  # native backtrace if anything below crashes (test helper, not product)
        ctypes.CDLL(bt).segv_bt_install()
    hip = _hip()
    saved = ecg.get_option(ecg.ECG_OPT_PROGRAM_CACHE)
    rng = np.random.default_rng(11)
    Bs = 4096
    blocks = torch.from_numpy(rng.integers(0, 256, (4, Bs), dtype=np.uint8)).cuda()
    host = blocks.cpu().numpy()
    mats = [[int(x) for x in rng.integers(1, 256, 4 * 2)] for _ in range(40)]
    outs = [torch.zeros((2, Bs), dtype=torch.uint8, device="cuda") for _ in mats]
    big = torch.empty((64, 14, 1 << 20), dtype=torch.uint8, device="cuda")
    ecg.fill_random(big, 0x5EED)
    M = ecg.reed_sol_vandermonde_coding_matrix(10, 4)
    torch.cuda.synchronize()
    handles = []
    try:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, 2)
        it = iter(zip(mats, outs))
        for rnd in range(6):
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            handles.append(s.value)
            # work queued on the caller stream, then calls whose program sets remember it
            ecg.encode_batch(10, 4, M, big[:, :10], big[:, 10:], stream=s.value)
            with ecg.batch():  # a scope on the caller stream (its flush orders after earlier flushes)
                for _ in range(2):
                    Mi, out = next(it)
                    ecg.dev_matrix_encode(4, 2, Mi, [blocks[j] for j in range(4)], [out[0], out[1]], Bs,
                                          stream=s.value)
            for _ in range(2):
                Mi, out = next(it)
                ecg.dev_matrix_encode(4, 2, Mi, [blocks[j] for j in range(4)], [out[0], out[1]], Bs,
                                      stream=s.value)
            if rnd % 2 == 0:  # destroyed with its work still queued (hipStreamDestroy waits for it)
                assert hip.hipStreamDestroy(s) == 0
            else:  # or idle, and a new stream (often the same handle) created before the evicting calls
                torch.cuda.synchronize()
                assert hip.hipStreamDestroy(s) == 0
                s2 = ctypes.c_void_p()
                assert hip.hipStreamCreate(ctypes.byref(s2)) == 0
                Mi, out = next(it)
                ecg.dev_matrix_encode(4, 2, Mi, [blocks[j] for j in range(4)], [out[0], out[1]], Bs,
                                      stream=s2.value)
                hip.hipStreamSynchronize(s2)
                assert hip.hipStreamDestroy(s2) == 0
            # evicting calls on torch's stream: every set used on the dead stream is retired here
            for _ in range(2):
                Mi, out = next(it)
                assert ecg.dev_matrix_encode(4, 2, Mi, [blocks[j] for j in range(4)], [out[0], out[1]],
                                             Bs) == 0
        torch.cuda.synchronize()
        left = ecg.lib().ecg_program_sets_retiring()
        print(f"stream handles {[hex(h) for h in handles]} ({len(set(handles))} distinct); "
              f"{left} evicted sets wait for a stream not seen again")
        used = len(mats) - sum(1 for _ in it)
        for Mi, out in list(zip(mats, outs))[:used]:
            want = [np.zeros(Bs, np.uint8) for _ in range(2)]
            oracle.jerasure_matrix_encode(4, 2, Mi, [host[j] for j in range(4)], want, Bs)
            assert np.array_equal(out.cpu().numpy(), np.stack(want))
        # the sets whose last stream was destroyed are freed by a reclaim (device synchronize), nothing else
        assert ecg.lib().ecg_program_sets_reclaim() == 0
    finally:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, saved)


def test_per_thread_stream_sets_are_covered_only_by_their_thread(ecg, oracle):
    """hipStreamPerThread is one handle value naming a different stream on every thread.
    Thread A builds program set P_A (one call, synchronized), queues ~90 ms of encodes on ITS per-thread
    stream, then calls P_A again; that launch, noted under the handle, waits behind the queue.  Thread B, on ITS per-thread stream, forces
    P_A's eviction (cache of 2) with twenty new programs of the same shape, synchronizing its own stream
    after each.  A cover recorded on B's stream would fire at once, P_A's tables would return to the pool,
    and B's next upload would overwrite them while A's call is still queued.  A's result must equal the
    oracle's; the library may cover P_A only from thread A (engine.hpp stream_key).  On the GPU this
    discriminates only when the two per-thread streams land on different hardware queues; the CPU harness
    (tools/tsan_host.sh sharedkey, tests/test_sanitize.py) checks the same scenario deterministically."""
    import threading

    import torch
    hip = _hip()
    PER_THREAD = 2  # hipStreamPerThread
    saved = ecg.get_option(ecg.ECG_OPT_PROGRAM_CACHE)
    rng = np.random.default_rng(23)
    Bs = 64 << 10
    blocks = torch.from_numpy(rng.integers(0, 256, (4, Bs), dtype=np.uint8)).cuda()
    host = blocks.cpu().numpy()
    mat_a = [int(x) for x in rng.integers(2, 256, 4 * 2)]
    mats_b = [[int(x) for x in rng.integers(2, 256, 4 * 2)] for _ in range(20)]
    out_a = torch.zeros((2, Bs), dtype=torch.uint8, device="cuda")
    outs_b = [torch.zeros((2, Bs), dtype=torch.uint8, device="cuda") for _ in mats_b]
    big = torch.empty((64, 14, 1 << 20), dtype=torch.uint8, device="cuda")
    ecg.fill_random(big, 0x7EED)
    M = ecg.reed_sol_vandermonde_coding_matrix(10, 4)
    torch.cuda.synchronize()
    queued, b_done, errors = threading.Event(), threading.Event(), []
    a_made, b_made, still_queued = threading.Event(), threading.Event(), []

    def thread_a():
        try:
            # the two per-thread streams are created back to back, so the runtime deals them to different
            # hardware queues (it hands new streams the queues in turn) and B's work does not wait behind A's
            assert hip.hipStreamQuery(PER_THREAD) == 0
            a_made.set()
            b_made.wait(60)
            # P_A built and uploaded first, so nothing but the queued launch below holds its tables
            ecg.dev_matrix_encode(4, 2, mat_a, [blocks[j] for j in range(4)], [out_a[0], out_a[1]], Bs,
                                  stream=PER_THREAD)
            assert hip.hipStreamSynchronize(PER_THREAD) == 0
            out_a.zero_()
            torch.cuda.synchronize()
            for _ in range(600):  # ~90 ms of work ahead of the call below, on A's per-thread stream
                ecg.encode_batch(10, 4, M, big[:, :10], big[:, 10:], stream=PER_THREAD)
            ecg.dev_matrix_encode(4, 2, mat_a, [blocks[j] for j in range(4)], [out_a[0], out_a[1]], Bs,
                                  stream=PER_THREAD)
            queued.set()
            b_done.wait(60)
            still_queued.append(hip.hipStreamQuery(PER_THREAD) != 0)  # A's call not yet run when B finished
            assert hip.hipStreamSynchronize(PER_THREAD) == 0
        except Exception as e:  # noqa: BLE001
            errors.append(e)
            queued.set()

    def thread_b():
        try:
            a_made.wait(60)
            assert hip.hipStreamQuery(PER_THREAD) == 0
            b_made.set()
            queued.wait(60)
            for Mi, out in zip(mats_b, outs_b):
                ecg.dev_matrix_encode(4, 2, Mi, [blocks[j] for j in range(4)], [out[0], out[1]], Bs, stream=PER_THREAD)
                assert hip.hipStreamSynchronize(PER_THREAD) == 0
        except Exception as e:  # noqa: BLE001
            errors.append(e)
        finally:
            b_done.set()

    try:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, 2)
        ta, tb = threading.Thread(target=thread_a), threading.Thread(target=thread_b)
        ta.start()
        tb.start()
        ta.join(120)
        tb.join(120)
        assert not errors, errors
        # whether the scenario could discriminate on this box: B's evictions ran while A's call was queued
        print(f"A's call still queued when B finished: {still_queued}")
        torch.cuda.synchronize()
        for Mi, out in [(mat_a, out_a)] + list(zip(mats_b, outs_b)):
            want = [np.zeros(Bs, np.uint8) for _ in range(2)]
            oracle.jerasure_matrix_encode(4, 2, Mi, [host[j] for j in range(4)], want, Bs)
            assert np.array_equal(out.cpu().numpy(), np.stack(want)), "a call on hipStreamPerThread read reused tables"
        assert ecg.lib().ecg_program_sets_reclaim() == 0
    finally:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, saved)


def test_graveyard_bound_frees_sets_of_streams_never_seen_again(ecg, oracle):
    """Evicted sets whose streams the library is never handed again cannot be covered (engine.hpp
    ProgramSet): they wait in the graveyard, which one device synchronize empties once it outgrows
    ECG_OPT_GRAVEYARD.  Forty per-request streams (all alive at once, so no handle is reused), each running
    two distinct programs once and never used again; with a cache of 2 and a graveyard of 3, the retiring
    count stays bounded and every result matches the oracle."""
    import ctypes

    import torch
    hip = _hip()
    saved = (ecg.get_option(ecg.ECG_OPT_PROGRAM_CACHE), ecg.get_option(ecg.ECG_OPT_GRAVEYARD))
    rng = np.random.default_rng(23)
    Bs = 4096
    blocks = torch.from_numpy(rng.integers(0, 256, (4, Bs), dtype=np.uint8)).cuda()
    host = blocks.cpu().numpy()
    torch.cuda.synchronize()
    try:
        assert ecg.lib().ecg_program_sets_reclaim() == 0
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, 2)
        ecg.set_option(ecg.ECG_OPT_GRAVEYARD, 3)
        peak = 0
        streams = []
        for _ in range(40):
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            streams.append(s)
        assert len({x.value for x in streams}) == 40
        for req, s in enumerate(streams):
            outs = []
            for j in range(2):
                Mi = [int(x) for x in rng.integers(1, 256, 8)]
                out = torch.zeros((2, Bs), dtype=torch.uint8, device="cuda")
                assert ecg.dev_matrix_encode(4, 2, Mi, [blocks[i] for i in range(4)], [out[0], out[1]], Bs,
                                             stream=s.value) == 0
                outs.append((Mi, out))
            hip.hipStreamSynchronize(s)
            for Mi, out in outs:
                want = [np.zeros(Bs, np.uint8) for _ in range(2)]
                oracle.jerasure_matrix_encode(4, 2, Mi, [host[i] for i in range(4)], want, Bs)
                assert np.array_equal(out.cpu().numpy(), np.stack(want)), req
            peak = max(peak, ecg.lib().ecg_program_sets_retiring())
        for s in streams:
            assert hip.hipStreamDestroy(s) == 0
        print(f"retiring peak {peak} with a graveyard of 3")
        assert peak <= 3 + 4, peak  # the bound, plus the sets evicted by the last miss and not yet swept
        assert ecg.lib().ecg_program_sets_reclaim() == 0
    finally:
        ecg.set_option(ecg.ECG_OPT_PROGRAM_CACHE, saved[0])
        ecg.set_option(ecg.ECG_OPT_GRAVEYARD, saved[1])
