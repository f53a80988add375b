#!/usr/bin/env python3
"""Stripe layouts x buffers for the config-2 encode (tuning tool, one process, interleaved rounds).

tools/placement_probe.py showed the encode moving 0.77 <-> 0.79 with WHICH stripe buffer it runs on (the
physical pages it got), so a layout compared on one buffer can win or lose by placement alone.  This
times every layout on each of several separate allocations in one process, so a layout's effect can be
told from the buffer's.  Layouts (block b of stripe s at base + s * SS + b * P):
  dense       P = 1 MiB,            SS = 14 P  (bench.py's [S][14][B])
  pitch+4K    P = 1 MiB + 4 KiB,    SS = 14 P
  pitch+64K   P = 1 MiB + 64 KiB,   SS = 14 P
  pitch+146K  P = 1 MiB + 146 KiB,  SS = 14 P  (the 14 blocks spread over one more 2 MiB page)
  spare       P = 1 MiB,            SS = 15 P  (one spare block per stripe, [S][15][B])
  stripe+2M   P = 1 MiB,            SS = 16 MiB (stripes on 16 MiB boundaries)
Prints, per layout, the median over all buffers and each buffer's median (algorithmic (k + m) B S bytes
per launch / t / 8 TB/s).
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

MiB, KiB = 1 << 20, 1 << 10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--buffers", type=int, default=3)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, MiB, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    layouts = {"dense": (B, n * B), "pitch+4K": (B + 4 * KiB, n * (B + 4 * KiB)),
               "pitch+64K": (B + 64 * KiB, n * (B + 64 * KiB)), "pitch+146K": (B + 146 * KiB, n * (B + 146 * KiB)),
               "spare": (B, (n + 1) * B), "stripe+2M": (B, 16 * MiB)}
    size = max((S - 1) * ss + (n - 1) * p + B for p, ss in layouts.values())
    bufs = [torch.empty(size, dtype=torch.uint8, device="cuda") for _ in range(a.buffers)]
    for b in bufs:
        ecg.fill_random(b.view(1, 1, size), 0xEC0DE)
    variants = []
    for bi, buf in enumerate(bufs):
        for name, (p, ss) in layouts.items():
            d = buf.as_strided((S, k, B), (ss, p, 1))
            c = buf.as_strided((S, m, B), (ss, p, 1), k * p)
            variants.append((name, bi, (lambda d=d, c=c: ecg.encode_batch(k, m, M, d, c))))
    times = {(v[0], v[1]): [] for v in variants}
    for _, _, fn in variants:
        fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, bi, fn in variants:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            evs[0].record()
            for i in range(a.reps):
                fn()
                evs[i + 1].record()
            torch.cuda.synchronize()
            times[(name, bi)] += [evs[i].elapsed_time(evs[i + 1]) for i in range(a.reps)]
    nbytes = S * n * B
    frac = lambda t: nbytes / (t * 1e-3) / 8e12  # noqa: E731
    out = {"buffers": [hex(b.data_ptr()) for b in bufs]}
    for name in layouts:
        per = [statistics.median(times[(name, bi)]) for bi in range(a.buffers)]
        allt = [t for bi in range(a.buffers) for t in times[(name, bi)]]
        out[name] = {"frac_median_all": round(frac(statistics.median(allt)), 4),
                     "frac_per_buffer": [round(frac(t), 4) for t in per]}
        print(f"{name:11s} all {out[name]['frac_median_all']:.4f}   per buffer "
              + " ".join(f"{x:.4f}" for x in out[name]["frac_per_buffer"]), flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
