#!/usr/bin/env python3
"""Config 5's wave encode vs the headline encode (tuning tool, one process, interleaved rounds).

bench.py's `config5` object encodes RS(10,4) 4 MiB stripes in waves of 1024 (56 GiB, the same bytes as
the headline's 4096 x 1 MiB launch) and measured 0.770-0.782 of HBM where the headline encode measured
0.790-0.794 on the same boxes.  This separates the candidate causes on one 56 GiB buffer viewed both ways:
  * block size: [4096][14][1 MiB] vs [1024][14][4 MiB], launched back to back;
  * what precedes the launch: the previous encode (back to back) vs the wave's regeneration kernel
    (fill_random over the whole wave, as encode_waves does);
  * grid map for the 4 MiB shape (auto = XCD-contiguous, stripe per XCD, linear) and columns per workgroup.
Each variant: `reps` HIP-event-timed launches per round, rounds interleaved; prints median / best and the
algorithmic HBM fraction ((k + m) B S / t / 8 TB/s).
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m = 10, 4
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    total = 4096 * n * (1 << 20)
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    ecg.fill_random(buf.view(4096, n, 1 << 20), 0xEC0DE)
    v1 = buf.view(4096, n, 1 << 20)
    v4 = buf.view(1024, n, 4 << 20)
    knobs = (ecg.ECG_OPT_GRID_MAP, ecg.ECG_OPT_COLS_PER_WG)
    saved = [ecg.get_option(o) for o in knobs]

    def enc(v):
        return lambda: ecg.encode_batch(k, m, M, v[:, :k], v[:, k:])

    variants = [  # (name, launch, pre (untimed, right before each timed launch) or None, options)
        ("1MiB x4096 back-to-back", enc(v1), None, {}),
        ("4MiB x1024 back-to-back", enc(v4), None, {}),
        ("1MiB x4096 after fill", enc(v1), lambda: ecg.fill_random(v1, 7), {}),
        ("4MiB x1024 after fill", enc(v4), lambda: ecg.fill_random(v4, 7), {}),
        ("4MiB x1024 map2", enc(v4), None, {ecg.ECG_OPT_GRID_MAP: 2}),
        ("4MiB x1024 map0", enc(v4), None, {ecg.ECG_OPT_GRID_MAP: 0}),
        ("4MiB x1024 cpw=256", enc(v4), None, {ecg.ECG_OPT_COLS_PER_WG: 256}),
    ]

    def setup(opts):
        for o, v in zip(knobs, saved):
            ecg.set_option(o, opts.get(o, v))

    times = {v[0]: [] for v in variants}
    for name, fn, pre, opts in variants:  # warm-up
        setup(opts)
        fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, fn, pre, opts in variants:
            setup(opts)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in evs:
                if pre:
                    pre()
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) for e0, e1 in evs]
    setup({})
    out = {}
    for name, *_ in variants:
        t = times[name]
        med, best = statistics.median(t), min(t)
        out[name] = {"median_ms": round(med, 3), "best_ms": round(best, 3),
                     "frac_median": round(total / (med * 1e-3) / 8e12, 4), "frac_best": round(total / (best * 1e-3) / 8e12, 4)}
        print(f"{name:26s} median {med:7.3f} ms ({out[name]['frac_median']:.4f})  best {best:7.3f} ms "
              f"({out[name]['frac_best']:.4f})", flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
