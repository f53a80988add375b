"""N>1 path on CPU: world_size-2 gloo processes run ecg_dist's sharding, barrier, max-reduce and
checksum all-gather exactly as bench.py does on GPUs.  The per-stripe coding work is done by the oracle
(CPU stand-in: this test covers the distributed logic, the kernels are covered by the GPU tests)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _encode_range(first, last, k, m, B, seed):
    from oracle import ref
    M = ref.reed_sol_vandermonde_coding_matrix(k, m)
    out = []
    for s in range(first, last):
        data = [ref.splitmix_bytes(seed, (s * (k + m) + j) * B // 8, B) for j in range(k)]
        coding = [np.zeros(B, np.uint8) for _ in range(m)]
        ref.jerasure_matrix_encode(k, m, M, data, coding, B)
        out.append(np.concatenate(coding))
    return np.concatenate(out) if out else np.zeros(0, np.uint8)


def _worker(rank, world, port, total, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import ecg_dist as D
    r = D.from_env()
    D.init(r, backend="gloo")
    k, m, B, seed = 6, 3, 256, 0xEC0DE
    first, last = D.stripe_range(total, r)
    D.barrier(r)
    par = _encode_range(first, last, k, m, B, seed)
    c = D.checksum64(torch.from_numpy(par))
    # device="cuda" as bench.py passes it: under gloo (bench's ECG_BENCH_SHARED_GPU rehearsal and these
    # tests) ecg_dist keeps the bookkeeping tensors on the host
    sums = D.gather_checksums(c, r, device="cuda")
    t = D.max_over_ranks(float(rank + 1), r, device="cuda")
    n = D.sum_over_ranks(float(last - first), r, device="cuda")
    plan = D.broadcast_ints([7, 1, 255, 0, 42] if rank == 0 else None, r, device="cuda")
    fl = D.gather_floats([rank, 0.25 * rank, last - first], r, device="cuda")  # bench's per-rank fractions
    D.barrier(r)
    q.put((rank, first, last, sums, t, n, plan, fl))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("total", [10, 3])
def test_two_rank_sharding_matches_single_process(total):
    sys.path[:0] = [os.path.join(ROOT, "erasure-codes-prototype_amd")]
    import ecg_dist as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    [p.start() for p in procs]
    res = sorted(q.get(timeout=120) for _ in procs)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    # ranges tile [0, total) contiguously
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == total
    # every rank saw the same gathered checksums; combined == single-process checksum
    assert res[0][3] == res[1][3]
    full = _encode_range(0, total, 6, 3, 256, 0xEC0DE)
    assert D.combine(res[0][3]) == D.checksum64(torch.from_numpy(full))
    # max over ranks of (rank+1) and the sum of processed stripes
    assert res[0][4] == res[1][4] == 2.0
    assert res[0][5] == res[1][5] == float(total)
    # the coding plan fanned out from rank 0
    assert res[0][6] == res[1][6] == [7, 1, 255, 0, 42]
    # every rank's float list, in rank order, on every rank
    want = [[0.0, 0.0, float(res[0][2] - res[0][1])], [1.0, 0.25, float(res[1][2] - res[1][1])]]
    assert res[0][7] == res[1][7] == want


def test_stripe_range_single_and_uneven():
    sys.path[:0] = [os.path.join(ROOT, "erasure-codes-prototype_amd")]
    import ecg_dist as D
    for total in (0, 1, 7, 8, 65536):
        for world in (1, 2, 3, 8):
            spans = [D.stripe_range(total, D.Rank(r, world, r)) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    assert D.data_word_offset(3, 14, 1 << 20) == 3 * 14 * (1 << 20) // 8


def _ring_worker(rank, world, port, S, chunk, q):
    """Cross-GPU partial decoding (ecg_dist.pipelined_ring_repair) with gloo and host tensors: rank r is
    the helper proxy for rank r + 1's stripes.  The partial arithmetic is the oracle's (CPU stand-in for
    the kernels); what is under test is the ring routing, the chunk pipeline and the wait points."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import ecg_dist as D
    from ecg_ring import azure_local_split
    from oracle import ec_ref as E
    from oracle import ref
    r = D.from_env()
    D.init(r, backend="gloo")
    B, n = 64, 16
    cp = E.CodingParameters(k=12, l=2, g=2, local_or_column=True)
    ec = E.ec_factory(E.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)  # local_or_column reaches the object here (handle_repair.cpp:14)
    cls_local = [e for e in range(n) if e not in (12, 13)]

    def stripe(gs):  # global stripe gs: 16 blocks
        data = [ref.splitmix_bytes(0xEC0DE, (gs * n + j) * B // 8, B) for j in range(12)]
        coding = E.zeros(4, B)
        ec.encode(data, coding, B)
        return data + coding

    def partial(blocks, e, which):
        surv, sets = azure_local_split(e)
        out = E.zeros(1, B)
        ec.encode_partial_blocks_for_decoding([blocks[b] for b in sets[which]], out, B, sets[which], surv, [e])
        return out[0]

    nxt = (rank + 1) % world
    send = torch.zeros((S, B), dtype=torch.uint8)
    recv = torch.zeros((S, B), dtype=torch.uint8)
    rebuilt = np.zeros((S, B), np.uint8)
    calls = []

    def helper(c0, c1):
        calls.append(("h", c0, c1))
        for i in range(c0, c1):
            gs = nxt * S + i
            send[i] = torch.from_numpy(partial(stripe(gs), cls_local[gs % 14], 0))

    def main(c0, c1):
        calls.append(("m", c0, c1))
        for i in range(c0, c1):
            gs = rank * S + i
            rebuilt[i] = partial(stripe(gs), cls_local[gs % 14], 1) ^ recv[i].numpy()

    D.pipelined_ring_repair(S, chunk, helper, main, send, recv, r)
    ok = all(np.array_equal(rebuilt[i], stripe(rank * S + i)[cls_local[(rank * S + i) % 14]]) for i in range(S))
    q.put((rank, ok, calls))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,S,chunk", [(2, 5, 2), (3, 4, 4), (8, 3, 2)])
def test_ring_partial_repair(world, S, chunk):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ring_worker, args=(r, world, port, S, chunk, q)) for r in range(world)]
    [p.start() for p in procs]
    res = sorted(q.get(timeout=120) for _ in procs)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok, _ in res), res
    # helper of chunk c + 1 is issued before the main kernel of chunk c
    spans = [(c, min(c + chunk, S)) for c in range(0, S, chunk)]
    want = [("h",) + spans[0]]
    for i in range(1, len(spans)):
        want += [("h",) + spans[i], ("m",) + spans[i - 1]]
    want.append(("m",) + spans[-1])
    assert res[0][2] == want


def _exchange_worker(rank, world, port, q):
    """ecg_dist.exchange with several shifted pairs in one batch (gloo, host tensors): pair d sends this
    rank's block d to rank - d and receives rank + d's block d; a shift that is a multiple of the world
    size stays on the rank (a copy)."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import ecg_dist as D
    r = D.from_env()
    D.init(r, backend="gloo")
    send = [torch.full((3, 8), 16 * rank + d, dtype=torch.uint8) for d in range(1, 5)]
    recv = [torch.zeros((3, 8), dtype=torch.uint8) for _ in range(4)]
    D.exchange([(send[d - 1], recv[d - 1], -d) for d in range(1, 5)], r).wait()
    ok = all(bool((recv[d - 1] == 16 * ((rank + d) % world) + d).all()) for d in range(1, 5))
    q.put((rank, ok))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_exchange_shifted_pairs(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    res = sorted(q.get(timeout=120) for _ in procs)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res), res


def test_ring_exchange_single_rank_and_shape_checks():
    sys.path[:0] = [os.path.join(ROOT, "erasure-codes-prototype_amd")]
    import ecg_dist as D
    r = D.Rank(0, 1, 0)
    a = torch.arange(12, dtype=torch.uint8).reshape(3, 4)
    b = torch.zeros_like(a)
    D.ring_exchange(a, b, r).wait()
    assert torch.equal(a, b)
    D.ring_exchange(a, a, r).wait()  # one rank, in place: nothing moves
    with pytest.raises(ValueError):
        D.ring_exchange(a, torch.zeros(4, 3, dtype=torch.uint8), r)
    with pytest.raises(ValueError):
        D.ring_exchange(a.t(), torch.zeros(4, 3, dtype=torch.uint8), r)
    with pytest.raises(ValueError):
        D.pipelined_ring_repair(3, 0, None, None, a, b, r)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_launcher_spawns_ranks(n):
    """`python bench.py --gpus N` outside torch.distributed starts N fresh rank processes itself (the
    driver's SCALE command) and relays rank 0's line with n_gpus = N.  --launch-check stops every rank
    after the gloo bookkeeping, before any GPU call."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    ranks = line["ranks"]
    assert sorted(r[0] for r in ranks) == list(range(n)) and sorted(r[1] for r in ranks) == list(range(n))
    assert len({r[2] for r in ranks}) == n and os.getpid() not in {r[2] for r in ranks}  # fresh processes


def test_bench_gpus_must_match_world():
    """Inside torch.distributed, --gpus N must equal WORLD_SIZE (a mismatched line would misreport n_gpus)."""
    import subprocess
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(extra)
    return env


def test_bench_stalled_rank_fails_within_dist_timeout():
    """A rank that never joins (injected: ECG_BENCH_TEST_STALL_RANK) must not hold the node: the other
    ranks' init_process_group gives up after ecg_dist's timeout (ECG_DIST_TIMEOUT_S), torch.distributed.run
    tears the job down, and bench.py exits non-zero -- well before the launcher's own watchdog."""
    import subprocess
    import time
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check",
                        "--timeout", "200"], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=_bench_env(ECG_BENCH_TEST_STALL_RANK="1", ECG_DIST_TIMEOUT_S="10"))
    took = time.time() - t0
    assert p.returncode not in (0, 124), (p.returncode, p.stderr[-2000:])
    assert took < 150, took
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_optional_section_deadline_keeps_the_line():
    """A sub-object of the line that hangs on one rank (injected: ECG_BENCH_TEST_STALL_OPTIONAL, the other
    rank waits for it in a collective) must not cost the line: every rank's optional-section deadline
    (ECG_BENCH_OPTIONAL_DEADLINE_S, below the collective timeout) fires first, rank 0 prints the
    line with an error object for the unfinished key, and every rank exits 0.  The collective timeout is
    generous (rank start-up -- importing torch -- can take long on a loaded machine) and the optional
    deadline is set below it explicitly."""
    import json
    import subprocess
    import time
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check",
                        "--timeout", "250"], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=_bench_env(ECG_BENCH_TEST_STALL_OPTIONAL="1", ECG_DIST_TIMEOUT_S="120",
                                      ECG_BENCH_OPTIONAL_DEADLINE_S="10"))
    took = time.time() - t0
    assert p.returncode == 0, (p.returncode, p.stderr[-2000:])
    assert took < 200, took
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    assert lines[0]["n_gpus"] == 2 and len(lines[0]["ranks"]) == 2
    assert "deadline" in lines[0]["optional"]["error"]
    assert lines[0].get("optional_deadline_hit") is True
    # without the stall the same section completes
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check",
                        "--timeout", "250"], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=_bench_env(ECG_DIST_TIMEOUT_S="120"))
    assert p.returncode == 0, p.stderr[-2000:]
    (line,) = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert line["optional"] == {"ok": True}
    assert "optional_deadline_hit" not in line


def test_deadline_disarms_and_fires():
    """ecg_dist.deadline: a body that finishes first disarms it; one that does not triggers on_expiry."""
    sys.path[:0] = [os.path.join(ROOT, "erasure-codes-prototype_amd")]
    import threading
    import time
    import ecg_dist as D
    fired = threading.Event()
    with D.deadline(0.5, fired.set):
        pass
    time.sleep(1.0)
    assert not fired.is_set()
    with D.deadline(0.2, fired.set):
        time.sleep(1.0)
    assert fired.is_set()
    with D.deadline(0, lambda: (_ for _ in ()).throw(AssertionError("no deadline at 0"))):
        time.sleep(0.1)


def test_bench_launcher_watchdog_kills_stuck_ranks():
    """The launcher's wall-clock watchdog (--timeout): with the ranks' own timeout far away, a stuck rank
    is killed with its whole process group and bench.py exits 124 shortly after the limit."""
    import subprocess
    import time
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check",
                        "--timeout", "15"], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=_bench_env(ECG_BENCH_TEST_STALL_RANK="1", ECG_DIST_TIMEOUT_S="3000"))
    took = time.time() - t0
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    assert 15 <= took < 120, took
    assert "terminating them" in p.stderr


def test_dist_init_passes_timeout(monkeypatch):
    """ecg_dist.init hands its timeout to init_process_group (rendezvous and every collective)."""
    sys.path[:0] = [os.path.join(ROOT, "erasure-codes-prototype_amd")]
    import datetime
    import ecg_dist as D
    seen = {}
    monkeypatch.setattr(D.dist, "is_initialized", lambda: False)
    monkeypatch.setattr(D.dist, "init_process_group", lambda backend, **kw: seen.update(kw, backend=backend))
    monkeypatch.setenv("ECG_DIST_TIMEOUT_S", "42")
    D.init(D.Rank(0, 2, 0), "nccl", device="cuda:0")
    assert seen == {"backend": "nccl", "timeout": datetime.timedelta(seconds=42), "device_id": "cuda:0"}
    D.init(D.Rank(0, 1, 0), "gloo")  # one rank: no process group at all


def test_bench_config34_cpu_baselines_verify():
    """bench.py's config3 / config4 CPU baselines (the oracle's run of the same per-stripe calls, reported
    beside the GPU forms) repair every sampled block correctly and report a rate; CPU only."""
    import types

    sys.path.insert(0, ROOT)
    import bench
    a = types.SimpleNamespace(cpu_seconds=0.4)
    c3 = bench.config3_cpu_baseline(a)
    assert c3["verified"] is True and c3["value"] > 0 and c3["repairs_per_s"] > 0, c3
    assert c3["kind"] == "port" and c3["cores"] >= 1
    c4 = bench.config4_cpu_baseline(a)
    assert c4["verified"] is True and c4["value"] > 0 and c4["merges_per_s"] > 0, c4
