#!/usr/bin/env python3
"""HBM rate by allocation, across most of the device memory (tuning tool, one process).

tools/placement_probe4.py: in alternate processes on one box the same code's encode runs at 0.77 or 0.79
and its decode at 0.765 or 0.79, following where the buffers land.  This allocates `--chunks` buffers of
`--gib` GiB each (most of the 288 GB), in allocation order, and times on every one of them the RS(10,4)
encode of the stripes that fit ([S][14][1 MiB]) and a 1 -> 1 copy through the engine (half the chunk to
the other half), interleaved over rounds.  A region of the physical memory that is slower shows up as a
run of chunks with a lower rate in every round.
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

MiB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=30)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B = 10, 4, MiB
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    size = a.gib << 30
    S = (size // (n * B)) // 8 * 8
    chunks = []
    for i in range(a.chunks):
        try:
            chunks.append(torch.empty(size, dtype=torch.uint8, device="cuda"))
        except RuntimeError:
            break
    print(f"{len(chunks)} chunks of {a.gib} GiB, {S} stripes each", flush=True)
    variants = []
    for i, c in enumerate(chunks):
        st = c[:S * n * B].view(S, n, B)
        ecg.fill_random(st, 0xEC0DE)
        half = (size // 2) // B
        src, dst = c[:half * B].view(half, 1, B), c[half * B:2 * half * B].view(half, 1, B)
        variants.append((i, "encode", lambda st=st: ecg.encode_batch(k, m, M, st[:, :k], st[:, k:]), S * n * B))
        variants.append((i, "copy", lambda s=src, d=dst: ecg.perform_addition_batch(1, 1, s, d), 2 * half * B))
    times = {(v[0], v[1]): [] for v in variants}
    for *_, fn, _ in variants:
        fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for i, kind, fn, _ in variants:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            evs[0].record()
            for r in range(a.reps):
                fn()
                evs[r + 1].record()
            torch.cuda.synchronize()
            times[(i, kind)] += [evs[r].elapsed_time(evs[r + 1]) for r in range(a.reps)]
    out = {"chunk_gib": a.gib, "addresses": [hex(c.data_ptr()) for c in chunks], "rows": []}
    for i in range(len(chunks)):
        row = {"chunk": i, "addr": hex(chunks[i].data_ptr())}
        for kind, nbytes in (("encode", S * n * B), ("copy", 2 * ((size // 2) // B) * B)):
            t = statistics.median(times[(i, kind)])
            row[kind] = round(nbytes / (t * 1e-3) / 8e12, 4)
        out["rows"].append(row)
        print(f"chunk {i:2d} {row['addr']}  encode {row['encode']:.4f}  copy {row['copy']:.4f}", flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
