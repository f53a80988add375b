#!/usr/bin/env python3
"""Kernel-variant microbenchmark for the encode/decode hot path (one process, interleaved rounds).

Each variant: HIP-event-timed launches over the BASELINE config-2 working set (RS(10,4), 1 MiB
blocks, 4096 stripes; 56 GiB, far beyond the 256 MiB Infinity Cache).  Prints achieved algorithmic
GB/s ((k+m)*B*S / t for encode, (k+1)*B*S for decode) and the fraction of the 8 TB/s HBM peak.
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


def timeit(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    fn()
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true", help="defaults only: encode, decode, copy, 10->1 xor")
    ap.add_argument("--only", default=None, help="run only the variants whose name contains this string")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, a.block, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    ones = [1] * (k * m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 1)
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    pats = [[e] for e in range(n)]
    data, coding = stripes[:, :k], stripes[:, k:]
    enc_bytes = S * n * B
    dec_bytes = S * (k + 1) * B

    def opt(nt=3, cpw=0, spec=0, gmap=3):
        def f():  # spec: historical argument (compile-time-k kernels were removed after r01)
            ecg.set_option(ecg.ECG_OPT_NT, nt)
            ecg.set_option(ecg.ECG_OPT_COLS_PER_WG, cpw)
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, gmap)
        return f

    variants = []
    if a.quick:
        flat = stripes.view(S * n, 1, B)
        halfS = S * n // 2
        src1, dst1 = flat[:halfS], flat[halfS:2 * halfS]
        variants += [
            ("encode RS(10,4) defaults", opt(3, 0, 0, 3), lambda: ecg.encode_batch(k, m, M, data, coding), enc_bytes),
            ("decode rot14 defaults", opt(3, 0, 0, 3),
             lambda: ecg.decode_batch(k, m, M, 1, pats, stripes, out=rebuilt, pattern_of_stripe=pos), dec_bytes),
            ("copy 1->1 defaults", opt(3, 0, 0, 3), lambda: ecg.perform_addition_batch(1, 1, src1, dst1),
             2 * halfS * B),
            ("xor 10->1 defaults", opt(3, 0, 0, 3), lambda: ecg.perform_addition_batch(10, 1, data, rebuilt),
             S * 11 * B)]
        variants += [
            ("decode rot14 in-place defaults", opt(3, 0, 0, 3),
             lambda: ecg.decode_batch(k, m, M, 1, pats, stripes, out=None, pattern_of_stripe=pos), dec_bytes),
            ("decode rot14 in-place map=1", opt(3, 0, 0, 1),
             lambda: ecg.decode_batch(k, m, M, 1, pats, stripes, out=None, pattern_of_stripe=pos), dec_bytes),
            ("decode rot14 in-place map=2", opt(3, 0, 0, 2),
             lambda: ecg.decode_batch(k, m, M, 1, pats, stripes, out=None, pattern_of_stripe=pos), dec_bytes)]
        for gmap in (1, 2):
            variants += [
                (f"encode map={gmap}", opt(3, 0, 0, gmap), lambda: ecg.encode_batch(k, m, M, data, coding), enc_bytes),
                (f"decode rot14 map={gmap}", opt(3, 0, 0, gmap),
                 lambda: ecg.decode_batch(k, m, M, 1, pats, stripes, out=rebuilt, pattern_of_stripe=pos), dec_bytes),
                (f"xor 10->1 map={gmap}", opt(3, 0, 0, gmap),
                 lambda: ecg.perform_addition_batch(10, 1, data, rebuilt), S * 11 * B)]
    if not a.quick:
        for gmap in (0, 1, 2):
            variants.append((f"encode GENERAL auto-cpw map={gmap}", opt(3, 0, 0, gmap),
                             lambda: ecg.encode_batch(k, m, M, data, coding), enc_bytes))
            variants.append((f"decode rot14 auto-cpw map={gmap}", opt(3, 0, 0, gmap),
                             lambda: ecg.decode_batch(k, m, M, 1, pats, stripes, out=rebuilt,
                                                      pattern_of_stripe=pos), dec_bytes))
        for cpw in (256, 512):
            variants.append((f"encode GENERAL cpw={cpw} map=1", opt(3, cpw, 0, 1),
                             lambda: ecg.encode_batch(k, m, M, data, coding), enc_bytes))
            variants.append((f"decode rot14 cpw={cpw} map=1", opt(3, cpw, 0, 1),
                             lambda: ecg.decode_batch(k, m, M, 1, pats, stripes, out=rebuilt,
                                                      pattern_of_stripe=pos), dec_bytes))
        for nt in (0, 1, 2):
            variants.append((f"encode GENERAL nt={nt}", opt(nt, 0, 0, 1),
                             lambda: ecg.encode_batch(k, m, M, data, coding), enc_bytes))
        variants.append(("encode BINARY(ones) defaults", opt(),
                         lambda: ecg.encode_batch(k, m, ones, data, coding), enc_bytes))
        flat = stripes.view(S * n, 1, B)
        halfS = S * n // 2
        src1, dst1 = flat[:halfS], flat[halfS:2 * halfS]
        for gmap in (0, 1):
            variants.append((f"copy 1->1 via engine map={gmap}", opt(3, 0, 0, gmap),
                             lambda: ecg.perform_addition_batch(1, 1, src1, dst1), 2 * halfS * B))
            variants.append((f"xor 10->1 map={gmap}", opt(3, 0, 0, gmap),
                             lambda: ecg.perform_addition_batch(10, 1, data, rebuilt), S * 11 * B))
    if a.only:
        variants = [v for v in variants if a.only in v[0]]
    res = {name: [] for name, *_ in variants}
    for r in range(a.rounds):
        for name, setup, fn, nbytes in variants:
            setup()
            ts = timeit(fn, a.reps)
            res[name] += [nbytes / (t * 1e-3) / 1e9 for t in ts]
    opt()()
    out = {}
    for name, *_ in variants:
        v = res[name]
        out[name] = {"median_GBps": round(statistics.median(v), 1), "max_GBps": round(max(v), 1),
                     "frac_of_8TBps": round(statistics.median(v) / 8000, 4)}
        print(f"{name:45s} median {statistics.median(v):8.1f} GB/s  max {max(v):8.1f}  "
              f"({statistics.median(v) / 8000 * 100:5.1f}% of 8 TB/s)", flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
