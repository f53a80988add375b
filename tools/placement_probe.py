#!/usr/bin/env python3
"""Does where a buffer lands in HBM move the config-2 kernels? (tuning tool, one process, interleaved rounds)

The same binary measures the separate-output decode at 0.765-0.797 and the encode at 0.777-0.794 of HBM
in different processes, sometimes inversely (tools/decode_sweep.py on two boxes, profiles/r03/decode_sweep/).
This allocates TWO stripe batches [4096][14][1 MiB] (S0, S1) and FOUR decode output buffers [4096][1][1 MiB]
(R0..R3, separated by spacer allocations of different sizes), then times, interleaved: the encode of S0 and
of S1, and the rotating single-erasure decode of S0 and S1 into each R.  If the spread follows the
buffers, placement (the physical pages a buffer got) is the variable, not the box or the kernel.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))

import torch  # noqa: E402

import ecg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, 1 << 20, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    pats = [[e] for e in range(n)]
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    bufs, spacers = {}, []
    bufs["S0"] = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    for i, gap in enumerate((0, 1 << 30, (2 << 20) + 4096, 7 << 30)):
        if gap:
            spacers.append(torch.empty(gap, dtype=torch.uint8, device="cuda"))
        bufs[f"R{i}"] = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    bufs["S1"] = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    for s in ("S0", "S1"):
        ecg.fill_random(bufs[s], 0xEC0DE)
        ecg.encode_batch(k, m, M, bufs[s][:, :k], bufs[s][:, k:])
    addr = {name: t.data_ptr() for name, t in bufs.items()}

    variants = []
    for s in ("S0", "S1"):
        st = bufs[s]
        variants.append((f"encode {s}", (lambda st=st: ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])), S * n * B))
        for r in ("R0", "R1", "R2", "R3"):
            out = bufs[r]
            variants.append((f"decode {s}->{r}", (lambda st=st, out=out: ecg.decode_batch(
                k, m, M, 1, pats, st, out=out, pattern_of_stripe=pos)), S * (k + 1) * B))
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
    out = {"addresses": {kk: hex(v) for kk, v in addr.items()}}
    print("addresses:", {kk: hex(v) for kk, v in addr.items()})
    for name, _, nbytes in variants:
        t = times[name]
        med, best = statistics.median(t), min(t)
        out[name] = {"median_ms": round(med, 3), "best_ms": round(best, 3),
                     "frac_median": round(nbytes / (med * 1e-3) / 8e12, 4)}
        print(f"{name:18s} median {med:7.3f} ms ({out[name]['frac_median']:.4f})  best {best:7.3f} ms", flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
