#!/usr/bin/env python3
"""Physically contiguous stripe buffers vs default allocations for the config-2 encode (tuning tool).

tools/placement_probe.py / layout_probe3.py: the encode runs at 0.77 or 0.79 of HBM depending on which
allocation the stripes live in, whatever the layout.  HIP can ask for physically contiguous device memory
(hipExtMallocWithFlags(..., hipDeviceMallocContiguous)).  If such buffers land consistently on the fast
side, an engine that owns its stripe arena can allocate it that way.  This allocates `--buffers` stripe
batches [S][14][1 MiB] each way (straight from the HIP runtime, not torch's allocator, so both kinds are
plain hipMalloc-family allocations), and times the encode on every buffer in interleaved rounds; it also
times the rotating single-erasure decode of each batch into one output buffer of the same kind.
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

MiB = 1 << 20
HIP_DEVICE_MALLOC_DEFAULT, HIP_DEVICE_MALLOC_CONTIGUOUS = 0x0, 0x4


class View:
    """The three things ecg's batch calls read from a tensor: shape, strides and the base pointer."""

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
    ap.add_argument("--buffers", type=int, default=2)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--maps", action="store_true", help="also the encode under grid map 2 (G = 1, 8, 64) and map 0")
    ap.add_argument("--offsets", default="", help="comma list of MiB: contiguous buffers get this much slack and the "
                    "encode also runs with the stripes shifted by each offset (physical = virtual offset there)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    k, m, B, S = 10, 4, MiB, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    pats = [[e] for e in range(n)]
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    size = S * n * B
    offs = [int(x) * MiB for x in a.offsets.split(",") if x]
    slack = max(offs, default=0)
    bufs, outs = {}, {}
    for kind, flag in (("default", HIP_DEVICE_MALLOC_DEFAULT), ("contiguous", HIP_DEVICE_MALLOC_CONTIGUOUS)):
        for i in range(a.buffers):
            p = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), size + (slack if flag else 0), flag)
            print(f"{kind}{i}: hipExtMallocWithFlags rc={rc} ptr={hex(p.value or 0)}", flush=True)
            if rc == 0:
                bufs[f"{kind}{i}"] = p.value
        p = ctypes.c_void_p()
        if hip.hipExtMallocWithFlags(ctypes.byref(p), S * B, flag) == 0:
            outs[kind] = p.value
    variants = []
    for name, ptr in bufs.items():
        st = View(ptr, (S, n, B), (n * B, B))
        ecg.fill_random(View(ptr, (size,), (1,)), 0xEC0DE)  # (the slack beyond `size` is encoded as is)
        d, c = View(ptr, (S, k, B), (n * B, B)), View(ptr + k * B, (S, m, B), (n * B, B))
        variants.append((f"encode {name}", (lambda d=d, c=c: ecg.encode_batch(k, m, M, d, c)), size))
        if a.maps:
            for gm, g in ((2, 1), (2, 8), (2, 64), (0, 1)):
                def enc(d=d, c=c, gm=gm, g=g):
                    ecg.set_option(ecg.ECG_OPT_GRID_MAP, gm)
                    ecg.set_option(ecg.ECG_OPT_MAP_GROUP, g)
                    try:
                        ecg.encode_batch(k, m, M, d, c)
                    finally:
                        ecg.set_option(ecg.ECG_OPT_GRID_MAP, 3)
                        ecg.set_option(ecg.ECG_OPT_MAP_GROUP, 1)
                variants.append((f"encode {name} map{gm} G={g}", enc, size))
        if name.startswith("contiguous"):
            for off in offs:
                dd, cc = View(ptr + off, (S, k, B), (n * B, B)), View(ptr + off + k * B, (S, m, B), (n * B, B))
                variants.append((f"encode {name} +{off // MiB}M", (lambda d=dd, c=cc: ecg.encode_batch(k, m, M, d, c)), size))
        kind = name.rstrip("0123456789")
        if kind in outs:
            o = View(outs[kind], (S, 1, B), (B, B))
            variants.append((f"decode {name}", (lambda st=st, o=o: ecg.decode_batch(
                k, m, M, 1, pats, st, out=o, pattern_of_stripe=pos)), S * (k + 1) * B))
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
    out = {}
    for name, _, nbytes in variants:
        med = statistics.median(times[name])
        out[name] = {"median_ms": round(med, 3), "frac_median": round(nbytes / (med * 1e-3) / 8e12, 4)}
        print(f"{name:32s} median {med:7.3f} ms ({out[name]['frac_median']:.4f})", flush=True)
    for ptr in list(bufs.values()) + list(outs.values()):
        hip.hipFree(ctypes.c_void_p(ptr))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
