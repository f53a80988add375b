"""Cross-GPU partial decoding on the GPU: ecg_ring's cross-GPU states (bench.py's
lrc-repair-ring / lrc-global-ring / pc-merge-ring), with the
helper-partial and fused main kernels running on cuda:0, checked byte for byte against the oracle.

The world-size-2 case runs two processes that share cuda:0 (the pool's boxes have one GPU) and move
the partials with gloo through host memory; on an 8-GPU node the same code moves them with RCCL over
xGMI.  RCCL refuses two ranks on one GPU, so its branch of ring_exchange runs here as one rank that is
its own RCCL peer (ecg_dist.init_self_p2p): the partials leave the helper's store and arrive in the main
proxy's through RCCL point-to-point ops, ordered with the kernels by the same stream waits.  Each rank's
repaired blocks are compared with the oracle's encode of the owner's stripes.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S, B, CHUNK = 20, 4096, 6


def _expected(owner):
    """Oracle: the lost block of each of the owner's S stripes (block-major splitmix layout of
    ecg_ring.ring_repair_state: block j of stripe i at word (owner * S * 17 + j * S + i) * B / 8)."""
    from oracle import ec_ref as E
    from oracle import ref
    cp = E.CodingParameters(k=12, l=2, g=2, local_or_column=True)
    ec = E.ec_factory(E.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    cls_local = [e for e in range(16) if e not in (12, 13)]
    out = []
    for i in range(S):
        data = [ref.splitmix_bytes(0xEC0DE, (owner * S * 17 + j * S + i) * B // 8, B) for j in range(12)]
        coding = E.zeros(4, B)
        ec.encode(data, coding, B)
        out.append((data + coding)[cls_local[(owner * S + i) % 14]])
    return np.stack(out)


def _run(r, self_p2p=False):
    import torch
    import ecg_ring
    step, rebuilt, _, _ = ecg_ring.ring_repair_state(r, S, B, CHUNK, self_p2p=self_p2p)
    rebuilt.zero_()
    step()
    torch.cuda.synchronize()
    return rebuilt[:, 0].cpu().numpy()


def _run_pc(r, self_p2p=False, S_=6, B_=8192):
    """Config 4's merge with the clusters on neighbouring ranks; returns whether every new row parity equals
    the XOR of the two old stripes' row blocks (recomputed with torch from regenerated stripes)."""
    import torch
    import ecg_ring
    step, out, expected = ecg_ring.pc_merge_ring_state(r, S_, B_, 2, self_p2p=self_p2p)
    out.zero_()
    step()
    torch.cuda.synchronize()
    return bool(torch.equal(out, expected(0, S_)))


def _worker(rank, world, port, q, glob=False):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import torch
        import ecg
        import ecg_dist as D
        torch.cuda.set_device(0)
        ecg.lib().ecg_set_device(0)
        r = D.from_env()
        D.init(r, "gloo")
        if glob == "pc":
            ok = _run_pc(r)
        else:
            got = _run_global(r) if glob else _run(r)
            ok = np.array_equal(got, _expected_global(rank) if glob else _expected(rank))
        torch.distributed.destroy_process_group()
        q.put((rank, ok, ""))
    except Exception as e:  # noqa: BLE001
        q.put((rank, False, repr(e)))


def test_ring_repair_one_rank(ecg, oracle):
    import ecg_dist as D
    assert np.array_equal(_run(D.Rank(0, 1, 0)), _expected(0))


@pytest.mark.parametrize("glob", [False, True, "pc"], ids=["local", "global", "pc-merge"])
def test_ring_repair_two_ranks_shared_gpu(ecg, oracle, glob):
    """Two ranks on cuda:0 (gloo moves the partials).  Global repairs: helpers at shifts 1 and 3 are the
    other rank, at 2 and 4 this rank itself (a local copy)."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, glob)) for r in range(2)]
    [p.start() for p in procs]
    res = sorted(q.get(timeout=100) for _ in procs)
    [p.join(timeout=30) for p in procs]
    assert [x[1] for x in res] == [True, True], res
    assert all(p.exitcode == 0 for p in procs)


def _self_p2p_worker(q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
    try:
        import torch
        import ecg
        import ecg_dist as D
        torch.cuda.set_device(0)
        ecg.lib().ecg_set_device(0)
        D.init_self_p2p(torch.device("cuda", 0))
        backend = torch.distributed.get_backend()
        got = _run(D.Rank(0, 1, 0), self_p2p=True)
        ok = np.array_equal(got, _expected(0))
        D.destroy()
        q.put((ok, backend, ""))
    except Exception as e:  # noqa: BLE001
        q.put((False, None, repr(e)))


def test_ring_repair_rccl_self_exchange(ecg, oracle):
    """The nccl branch of ring_exchange on hardware: one rank, its own RCCL peer, partials through RCCL."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_self_p2p_worker, args=(q,))
    p.start()
    ok, backend, err = q.get(timeout=100)
    p.join(timeout=30)
    assert ok, err
    assert backend == "nccl"
    assert p.exitcode == 0


def _expected_global(owner, S_=S):
    """Oracle: the lost global parity 12 + (owner * S + i) % 2 of each of the owner's stripes
    (ecg_ring.global_ring_state, same block-major splitmix layout as _expected)."""
    from oracle import ec_ref as E
    from oracle import ref
    cp = E.CodingParameters(k=12, l=2, g=2, local_or_column=True)
    ec = E.ec_factory(E.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    out = []
    for i in range(S_):
        data = [ref.splitmix_bytes(0xEC0DE, (owner * S_ * 17 + j * S_ + i) * B // 8, B) for j in range(12)]
        coding = E.zeros(4, B)
        ec.encode(data, coding, B)
        out.append(coding[(owner * S_ + i) % 2])
    return np.stack(out)


def _run_global(r, self_p2p=False):
    import torch
    import ecg_ring
    step, rebuilt, _, _ = ecg_ring.global_ring_state(r, S, B, CHUNK, self_p2p=self_p2p)
    rebuilt.zero_()
    step()
    torch.cuda.synchronize()
    return rebuilt[:, 0].cpu().numpy()


def test_global_ring_repair_one_rank(ecg, oracle):
    import ecg_dist as D
    assert np.array_equal(_run_global(D.Rank(0, 1, 0)), _expected_global(0))


def _global_self_p2p_worker(q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
    try:
        import torch
        import ecg
        import ecg_dist as D
        torch.cuda.set_device(0)
        ecg.lib().ecg_set_device(0)
        D.init_self_p2p(torch.device("cuda", 0))
        got = _run_global(D.Rank(0, 1, 0), self_p2p=True)
        ok = np.array_equal(got, _expected_global(0))
        D.destroy()
        q.put((ok, ""))
    except Exception as e:  # noqa: BLE001
        q.put((False, repr(e)))


def test_global_ring_repair_rccl_self_exchange(ecg, oracle):
    """Four helper partials per repair, all four through RCCL (rank 0 its own peer), vs the oracle."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_global_self_p2p_worker, args=(q,))
    p.start()
    ok, err = q.get(timeout=100)
    p.join(timeout=30)
    assert ok, err
    assert p.exitcode == 0


def test_pc_merge_ring_one_rank(ecg):
    import ecg_dist as D
    assert _run_pc(D.Rank(0, 1, 0))


def _pc_self_p2p_worker(q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
    try:
        import torch
        import ecg
        import ecg_dist as D
        torch.cuda.set_device(0)
        ecg.lib().ecg_set_device(0)
        D.init_self_p2p(torch.device("cuda", 0))
        ok = _run_pc(D.Rank(0, 1, 0), self_p2p=True)
        D.destroy()
        q.put((ok, ""))
    except Exception as e:  # noqa: BLE001
        q.put((False, repr(e)))


def test_pc_merge_ring_rccl_self_exchange(ecg):
    """Config 4's merge partials (5 rows per merge) through RCCL, rank 0 its own peer."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_pc_self_p2p_worker, args=(q,))
    p.start()
    ok, err = q.get(timeout=100)
    p.join(timeout=30)
    assert ok, err
    assert p.exitcode == 0
