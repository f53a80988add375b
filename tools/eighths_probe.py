#!/usr/bin/env python3
"""Is a slow stripe buffer slow everywhere, or in one part?  (tuning tool, one process)

Grid map 1 gives each XCD a contiguous eighth of the chunk list, so a launch ends when the slowest XCD's
eighth is done.  If a buffer's slowness (0.77 vs 0.79-0.80 of HBM, profiles/r03/placement/) sat in part of
its pages, the eighth on those pages would hold the whole launch while map 2 (stripes dealt round-robin
to the XCDs) would average it out.  This times, on each of `--buffers` allocations: the full encode under
map 1 and map 2, and each eighth of its stripes encoded on its own (a full-chip launch over S / 8 stripes).
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
    ap.add_argument("--buffers", type=int, default=3)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, 1 << 20, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    bufs = [torch.empty((S, n, B), dtype=torch.uint8, device="cuda") for _ in range(a.buffers)]
    for b in bufs:
        ecg.fill_random(b, 0xEC0DE)

    def enc(st, gm=3):
        def f():
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, gm)
            ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, 3)
        return f

    E = S // 8
    variants = []
    for bi, b in enumerate(bufs):
        variants.append((bi, "map1", enc(b), S * n * B))
        variants.append((bi, "map2", enc(b, 2), S * n * B))
        for e in range(8):
            variants.append((bi, f"eighth{e}", enc(b[e * E:(e + 1) * E]), E * n * B))
    times = {(v[0], v[1]): [] for v in variants}
    for *_, fn, _ in variants:
        fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for bi, name, fn, _ in variants:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            evs[0].record()
            for i in range(a.reps):
                fn()
                evs[i + 1].record()
            torch.cuda.synchronize()
            times[(bi, name)] += [evs[i].elapsed_time(evs[i + 1]) for i in range(a.reps)]
    res = {}
    for bi in range(a.buffers):
        row = {}
        for b2, name, _, nbytes in variants:
            if b2 == bi:
                row[name] = round(nbytes / (statistics.median(times[(bi, name)]) * 1e-3) / 8e12, 4)
        res[f"buffer{bi}"] = row
        print(f"buffer{bi}: map1 {row['map1']:.4f} map2 {row['map2']:.4f}  eighths "
              + " ".join(f"{row[f'eighth{e}']:.4f}" for e in range(8)), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
