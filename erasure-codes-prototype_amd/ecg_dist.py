"""Stripe sharding across GPUs: one process per GPU, no data-path collective.

Stripes are independent (the proxy loops stripes with no cross-stripe state, proxy.cpp:312-399), so a
batch of S_total stripes is partitioned into contiguous ranges, one per rank.  torch.distributed is
used only around the data path: a broadcast of the coding plan from rank 0 (coding matrix, erasure
patterns) before it, a barrier before/after the timed region, a MAX of elapsed times, a SUM of
processed bytes and an all-gather of per-rank 64-bit parity checksums for a bit-exact verdict.
Backend "nccl" (RCCL over xGMI) on GPUs, "gloo" in CPU tests.

The one real exchange step is cross-GPU partial decoding ("clusters -> GPUs"): a
helper proxy's partial block travels to the main proxy, which XOR-adds it to its own partial
(help_repair -> main_repair, handle_repair.cpp:249-384).  RCCL has no XOR reduction, so the partials
move point to point (`ring_exchange`, one xGMI link per rank pair) and the addition runs in the main
rank's fused repair kernel; `pipelined_ring_repair` overlaps chunk c's transfer with the kernels of
the chunks around it.
"""
from __future__ import annotations

import contextlib
import datetime
import os
import threading
from dataclasses import dataclass

import torch
import torch.distributed as dist

_MASK64 = (1 << 64) - 1


@dataclass
class Rank:
    rank: int
    world: int
    local: int

    @property
    def distributed(self):
        return self.world > 1


def from_env() -> Rank:
    return Rank(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                int(os.environ.get("LOCAL_RANK", "0")))


_BACKEND = None
# One rank exchanging with itself over RCCL (init_self_p2p): the ring's send / receive then go through RCCL
# point to point (a copy on the one GPU) instead of staying in place, so a one-GPU box runs the exact nccl
# code path of ring_exchange -- P2P ops, RCCL's stream, the current stream waiting on it -- that the
# N > 1 ring runs over xGMI.
_SELF_P2P = False

# Seconds a rank waits in rendezvous or in any collective before it fails (ECG_DIST_TIMEOUT_S).  A rank
# that never joins, or an RCCL communicator that never forms, then ends the run with an error instead of
# holding the node: init_process_group raises once the store rendezvous times out, and a collective that
# does not complete within it aborts the communicator (torch's watchdog).
DEFAULT_TIMEOUT_S = 300.0


def timeout_s() -> float:
    return float(os.environ.get("ECG_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))


@contextlib.contextmanager
def deadline(seconds: float, on_expiry):
    """Run the body; if it has not finished `seconds` after entry, call on_expiry() from a watchdog thread.
    on_expiry must end the process (os._exit): the body may be stuck inside a collective that no Python
    code can interrupt.  Finishing first (normally or by an exception) disarms it.  seconds <= 0: no
    deadline.  Every rank arms its own, so a section that hangs on one rank ends on all of them."""
    if seconds is None or seconds <= 0:
        yield
        return
    done = threading.Event()

    def watch():
        if not done.wait(seconds):
            on_expiry()

    t = threading.Thread(target=watch, name="ecg-deadline", daemon=True)
    t.start()
    try:
        yield
    finally:
        done.set()


def init(r: Rank, backend: str = "nccl", device=None) -> None:
    global _BACKEND
    _BACKEND = backend
    if r.distributed and not dist.is_initialized():
        kw = {"timeout": datetime.timedelta(seconds=timeout_s())}
        if device is not None:
            kw["device_id"] = device
        dist.init_process_group(backend, **kw)


def init_self_p2p(device) -> None:
    """A world-size-1 RCCL process group on `device` (127.0.0.1 rendezvous on a free port) whose ring
    exchange sends to and receives from rank 0 itself; undo with destroy()."""
    global _BACKEND, _SELF_P2P
    if dist.is_initialized():
        raise RuntimeError("init_self_p2p: a process group already exists")
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=timeout_s()), device_id=device)
    _BACKEND, _SELF_P2P = "nccl", True


def destroy() -> None:
    global _SELF_P2P
    if dist.is_initialized():
        dist.destroy_process_group()
    _SELF_P2P = False


def stripe_range(total: int, r: Rank) -> tuple[int, int]:
    """Contiguous [first, last) stripes of rank r; sizes differ by at most one."""
    base, extra = divmod(total, r.world)
    first = r.rank * base + min(r.rank, extra)
    return first, first + base + (1 if r.rank < extra else 0)


def data_word_offset(first_stripe: int, n_blocks: int, block_size: int) -> int:
    """splitmix64 word offset of a rank's first stripe, so every rank generates the bytes the global
    batch would hold (a stripe's bytes do not depend on how the batch is sharded)."""
    return first_stripe * n_blocks * block_size // 8


def barrier(r: Rank) -> None:
    if r.distributed:
        dist.barrier()


def _dev(device):
    return "cpu" if _BACKEND == "gloo" else device  # gloo collectives run on host tensors


def _reduce(value: float, r: Rank, op, device) -> float:
    if not r.distributed:
        return value
    device = _dev(device)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(value: float, r: Rank, device="cpu") -> float:
    return _reduce(value, r, dist.ReduceOp.MAX, device)


def sum_over_ranks(value: float, r: Rank, device="cpu") -> float:
    return _reduce(value, r, dist.ReduceOp.SUM, device)


def broadcast_ints(vals, r: Rank, device="cpu", src: int = 0) -> list[int]:
    """Fan out a small integer list (coding matrix, erasure patterns) from rank `src` to every rank;
    other ranks pass None.  The only data-independent exchange before the timed region."""
    if not r.distributed:
        return list(vals)
    n = torch.tensor([len(vals) if r.rank == src else 0], dtype=torch.int64, device=_dev(device))
    dist.broadcast(n, src)
    t = (torch.tensor(list(vals), dtype=torch.int64, device=_dev(device)) if r.rank == src
         else torch.zeros(int(n.item()), dtype=torch.int64, device=_dev(device)))
    dist.broadcast(t, src)
    return [int(x) for x in t.tolist()]


def checksum64(t: torch.Tensor) -> int:
    """Order-independent 64-bit checksum of a uint8 buffer: sum of its little-endian 8-byte words mod
    2^64 (the buffer length must be a multiple of 8)."""
    words = t.reshape(-1).view(torch.int64)
    return int(words.sum().item()) & _MASK64


def gather_floats(vals, r: Rank, device="cpu") -> list[list[float]]:
    """All-gather a short list of floats from every rank: result[q] is rank q's list (same length on
    every rank).  Per-rank HBM fractions and times for the bench line, after the timed region."""
    vals = [float(v) for v in vals]
    if not r.distributed:
        return [vals]
    t = torch.tensor(vals, dtype=torch.float64, device=_dev(device))
    out = [torch.zeros_like(t) for _ in range(r.world)]
    dist.all_gather(out, t)
    return [[float(x) for x in o.tolist()] for o in out]


def combine(checksums) -> int:
    return sum(int(c) for c in checksums) & _MASK64


def gather_checksums(c: int, r: Rank, device="cpu") -> list[int]:
    if not r.distributed:
        return [c]
    v = c if c < (1 << 63) else c - (1 << 64)  # carry the 64-bit pattern in a signed tensor
    t = torch.tensor([v], dtype=torch.int64, device=_dev(device))
    out = [torch.zeros_like(t) for _ in range(r.world)]
    dist.all_gather(out, t)
    return [int(x.item()) & _MASK64 for x in out]


def exchange(pairs, r: Rank):
    """Post, for every (send, recv, shift) in `pairs`: send -> rank + shift and recv <- rank - shift (mod
    world), all in one batch of RCCL point-to-point ops; returns a handle whose wait() makes every recv
    usable (on nccl: the current stream waits for RCCL's).  send and recv of a pair are contiguous tensors of
    one shape.  A pair whose peer is this rank itself (one rank, or a shift that is a multiple of the world
    size: helper and main proxy on the same GPU) is a local copy -- unless init_self_p2p made rank 0 its own
    RCCL peer, when it goes through RCCL like any other pair."""
    for send, recv, _ in pairs:
        if send.shape != recv.shape or not send.is_contiguous() or not recv.is_contiguous():
            raise ValueError("exchange: send and recv must be contiguous tensors of one shape")
    ops, staged = [], []
    for i, (send, recv, shift) in enumerate(pairs):
        dst, src = (r.rank + shift) % r.world, (r.rank - shift) % r.world
        if dst == r.rank and not _SELF_P2P:
            if recv.data_ptr() != send.data_ptr():
                recv.copy_(send)
            continue
        if _BACKEND == "gloo" and send.is_cuda:  # gloo moves host tensors: stage the pair through host memory
            hs = send.cpu()
            hr = torch.empty_like(hs)
            staged.append((hr, recv))
            send, recv = hs, hr
        # one tag per pair: gloo matches a recv to the send of the same pair index on the peer
        ops += [dist.P2POp(dist.isend, send, dst, tag=i), dist.P2POp(dist.irecv, recv, src, tag=i)]
    works = dist.batch_isend_irecv(ops) if ops else []

    class _Works:
        def wait(self):
            for w in works:
                w.wait()
            for hr, recv in staged:
                recv.copy_(hr)
    return _Works()


def ring_exchange(send: torch.Tensor, recv: torch.Tensor, r: Rank):
    """Post send -> rank + 1 and recv <- rank - 1 (mod world) of two contiguous tensors of one shape;
    returns a handle whose wait() makes the data usable (on nccl: the current stream waits for RCCL's).
    With one rank the block stays where it is (recv = send), unless init_self_p2p made rank 0 its own
    RCCL peer."""
    return exchange([(send, recv, 1)], r)


def pipelined_ring_repair(n_stripes: int, chunk: int, helper, main, send, recv, r: Rank, xchg=None) -> None:
    """Cross-GPU partial decoding over a ring of ranks, chunk by chunk.

    Rank r is the helper proxy for the next rank's stripes and the main proxy for its own; stripe i's
    helper partial is send[i] here and recv[i] on rank r + 1.  For every chunk [c0, c1):
      helper(c0, c1)  -- launch the helper-partial kernel writing send[c0:c1]
      ring_exchange   -- send[c0:c1] -> rank + 1, recv[c0:c1] <- rank - 1 (queued behind the kernel)
      main(c0, c1)    -- after the chunk arrived: the main rank's fused kernel (own partial + addition)
    The main kernel of chunk c is issued after the helper kernel and the transfer of chunk c + 1, so
    transfers run back to back while the kernels fill the gaps.  xchg(c0, c1), when given, replaces the
    single ring exchange (e.g. several helpers per stripe: one exchange() of several shifted pairs)."""
    if chunk < 1:
        raise ValueError("chunk must be >= 1")
    spans = [(c, min(c + chunk, n_stripes)) for c in range(0, n_stripes, chunk)]
    pending = None
    for c0, c1 in spans:
        helper(c0, c1)
        h = xchg(c0, c1) if xchg is not None else ring_exchange(send[c0:c1], recv[c0:c1], r)
        if pending is not None:
            pending[0].wait()
            main(*pending[1])
        pending = (h, (c0, c1))
    if pending is not None:
        pending[0].wait()
        main(*pending[1])
