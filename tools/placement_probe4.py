#!/usr/bin/env python3
"""Decode output in the stripes' own allocation vs a separate allocation (tuning tool, one process).

bench.py allocates the rebuilt blocks [S][1][B] as their own tensor after the stripes.  Where that
buffer's pages land sets the decode at 0.74-0.83 of HBM (tools/placement_probe.py).  This times, in one
process and interleaved, the bench's arrangement (stripes, then a separate output tensor) against one
allocation holding both ([stripes | outputs], outputs right after the last stripe), each on its own
stripe batch, plus the encode of both batches.  Run it in several processes to sample placements.
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, 1 << 20, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    pats = [[e] for e in range(n)]
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    # bench.py's arrangement
    sep_st = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    sep_out = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    # one allocation: stripes, then the outputs
    arena = torch.empty(S * (n + 1) * B, dtype=torch.uint8, device="cuda")
    one_st = arena[:S * n * B].view(S, n, B)
    one_out = arena[S * n * B:].view(S, 1, B)
    for st in (sep_st, one_st):
        ecg.fill_random(st, 0xEC0DE)
        ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])
    variants = [
        ("encode separate", lambda: ecg.encode_batch(k, m, M, sep_st[:, :k], sep_st[:, k:]), S * n * B),
        ("decode separate", lambda: ecg.decode_batch(k, m, M, 1, pats, sep_st, out=sep_out, pattern_of_stripe=pos),
         S * (k + 1) * B),
        ("encode one-alloc", lambda: ecg.encode_batch(k, m, M, one_st[:, :k], one_st[:, k:]), S * n * B),
        ("decode one-alloc", lambda: ecg.decode_batch(k, m, M, 1, pats, one_st, out=one_out, pattern_of_stripe=pos),
         S * (k + 1) * B),
    ]
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
        out[name] = round(nbytes / (med * 1e-3) / 8e12, 4)
    print(json.dumps(out), flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
