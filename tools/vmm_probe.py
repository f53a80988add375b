#!/usr/bin/env python3
"""Stripe arenas from torch's allocator vs HIP virtual-memory arenas (tuning tool, one process).

The encode runs at 0.77 or 0.79-0.80 of HBM depending on the allocation (profiles/r03/placement/).  This
times the config-2 encode and the rotating single-erasure decode (outputs in the same arena, after the
stripes) on arenas of S * 15 * 1 MiB made four ways, interleaved over rounds:
  torch          torch.empty (hipMalloc through the caching allocator)
  vmm a2M        hipMemAddressReserve aligned to 2 MiB, one physical handle (tools/vmm_probe.cpp)
  vmm a1G        reservation aligned to 1 GiB, one physical handle
  vmm a1G c1G    reservation aligned to 1 GiB, 1 GiB physical handles
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))

import torch  # noqa: E402

import ecg  # noqa: E402

MiB, GiB = 1 << 20, 1 << 30


class View:
    def __init__(self, ptr, shape, strides):
        self.ptr, self.shape, self._st = ptr, shape, strides

    def data_ptr(self):
        return self.ptr

    def stride(self, i):
        return self._st[i]

    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libvmm_probe.so"))
    L.vmm_alloc.restype = ctypes.c_void_p
    L.vmm_alloc.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
    L.vmm_free.argtypes = [ctypes.c_void_p]
    gmin, grec = ctypes.c_size_t(), ctypes.c_size_t()
    print("granularity", L.vmm_granularity(ctypes.byref(gmin), ctypes.byref(grec)), gmin.value, grec.value, flush=True)
    k, m, B, S = 10, 4, MiB, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    pats = [[e] for e in range(n)]
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    size = S * (n + 1) * B  # stripes, then the outputs
    size = (size + GiB - 1) // GiB * GiB
    arenas, keep = {}, []
    t = torch.empty(size, dtype=torch.uint8, device="cuda")
    keep.append(t)
    arenas["torch"] = t.data_ptr()
    for name, align, chunk in (("vmm a2M", 2 * MiB, 0), ("vmm a1G", GiB, 0), ("vmm a1G c1G", GiB, GiB)):
        p = L.vmm_alloc(size, align, chunk)
        print(f"{name}: {hex(p or 0)}", flush=True)
        if p:
            arenas[name] = p
    variants = []
    for name, p in arenas.items():
        st = View(p, (S, n, B), (n * B, B))
        out = View(p + S * n * B, (S, 1, B), (B, B))
        ecg.fill_random(View(p, (S * n * B,), (1,)), 0xEC0DE)
        d, c = View(p, (S, k, B), (n * B, B)), View(p + k * B, (S, m, B), (n * B, B))
        ecg.encode_batch(k, m, M, d, c)
        variants.append((f"encode {name}", lambda d=d, c=c: ecg.encode_batch(k, m, M, d, c), S * n * B))
        variants.append((f"decode {name}", lambda st=st, o=out: ecg.decode_batch(k, m, M, 1, pats, st, out=o,
                                                                                  pattern_of_stripe=pos), S * (k + 1) * B))
    times = {v[0]: [] for v in variants}
    for _, fn, _ in variants:
        fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, fn, _ in variants:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            evs[0].record()
            for i in range(a.reps):
                fn()
                evs[i + 1].record()
            torch.cuda.synchronize()
            times[name] += [evs[i].elapsed_time(evs[i + 1]) for i in range(a.reps)]
    res = {}
    for name, _, nbytes in variants:
        med = statistics.median(times[name])
        res[name] = round(nbytes / (med * 1e-3) / 8e12, 4)
    print(json.dumps(res), flush=True)
    for name, p in arenas.items():
        if name != "torch":
            L.vmm_free(ctypes.c_void_p(p))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
