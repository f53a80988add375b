#!/usr/bin/env python3
"""Does RCCL run two ranks on ONE GPU (the pool's boxes have one)?  If it does, the nccl branch of
ecg_dist.ring_exchange can be exercised here: each rank sends a tensor to the next rank and receives from
the previous one over RCCL point to point, and an all-reduce checks the bookkeeping.  Launch with
torch.distributed.run --nproc-per-node 2; every rank uses cuda:0.  Bounded by ECG_DIST_TIMEOUT_S."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
import torch  # noqa: E402

import ecg_dist as D  # noqa: E402

r = D.from_env()
torch.cuda.set_device(0)
t0 = time.time()
try:
    D.init(r, "nccl", device=torch.device("cuda", 0))
    x = torch.full((4,), float(r.rank + 1), device="cuda")
    torch.distributed.all_reduce(x)
    send = torch.full((1 << 20,), r.rank + 7, dtype=torch.uint8, device="cuda")
    recv = torch.zeros_like(send)
    D.ring_exchange(send, recv, r).wait()
    torch.cuda.synchronize()
    prev = (r.rank - 1) % r.world
    ok = bool((recv == prev + 7).all()) and x[0].item() == sum(range(1, r.world + 1))
    print(f"rank {r.rank}: all_reduce {x[0].item()}, ring_exchange received {int(recv[0])} from rank {prev}: "
          f"{'OK' if ok else 'WRONG'} ({time.time() - t0:.1f} s)", flush=True)
    torch.distributed.destroy_process_group()
    sys.exit(0 if ok else 1)
except Exception as e:  # noqa: BLE001
    print(f"rank {r.rank}: {type(e).__name__}: {str(e)[:300]}", flush=True)
    sys.exit(3)
