#!/usr/bin/env python3
"""Grid-map sweep for the config-2 encode and decode (tuning tool, one process, interleaved rounds).

Grid map 1 gives each XCD group a contiguous eighth of the chunk list; grid map 2 deals runs of G adjacent
stripes to the XCD groups round-robin (ECG_OPT_MAP_GROUP = G; G = 1 is stripe s on group s % 8, G = S / 8
is map 1 up to chunk order).  So G sets how far apart in HBM the stripes the 8 XCDs work on at one time
are: G * (k + m) * B bytes.  Prints, per variant, the median and best HIP-event launch time over all
rounds and the algorithmic fraction of the 8 TB/s peak.
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
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--groups", default="1,2,4,8,16,32,64,128,256,512")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, a.block, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 1)
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    pats = [[e] for e in range(n)]
    groups = [int(g) for g in a.groups.split(",")]

    def enc():
        ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])

    def dec():
        ecg.decode_batch(k, m, M, 1, pats, stripes, out=rebuilt, pattern_of_stripe=pos)

    variants = [("encode map1", enc, 1, 1, S * n * B), ("decode map1", dec, 1, 1, S * (k + 1) * B)]
    for g in groups:
        variants.append((f"encode map2 G={g}", enc, 2, g, S * n * B))
        variants.append((f"decode map2 G={g}", dec, 2, g, S * (k + 1) * B))
    times = {v[0]: [] for v in variants}
    ref = None
    for rnd in range(a.rounds):
        order = variants if rnd % 2 == 0 else variants[::-1]
        for name, fn, gm, g, _ in order:
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, gm)
            ecg.set_option(ecg.ECG_OPT_MAP_GROUP, g)
            fn()  # warm (no idle gap before the timed launches)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) for e0, e1 in ev]
        if rnd == 0:  # every map writes the same bytes
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, 3)
            ecg.set_option(ecg.ECG_OPT_MAP_GROUP, 1)
            ref = stripes[:, k:].clone()
    for gm, g in ((2, 7), (2, 64), (1, 1)):
        ecg.set_option(ecg.ECG_OPT_GRID_MAP, gm)
        ecg.set_option(ecg.ECG_OPT_MAP_GROUP, g)
        stripes[:, k:].fill_(0x5A)
        enc()
        torch.cuda.synchronize()
        assert torch.equal(stripes[:, k:], ref), f"map {gm} G={g}: parities differ"
    ecg.set_option(ecg.ECG_OPT_GRID_MAP, 3)
    ecg.set_option(ecg.ECG_OPT_MAP_GROUP, 1)
    res = {}
    for name, _, _, _, nbytes in variants:
        t = times[name]
        med, best = statistics.median(t), min(t)
        res[name] = {"median_ms": round(med, 3), "best_ms": round(best, 3),
                     "frac_median": round(nbytes / (med * 1e-3) / 8e12, 4), "frac_best": round(nbytes / (best * 1e-3) / 8e12, 4)}
        print(f"{name:24s} median {med:7.3f} ms  best {best:7.3f} ms  frac {res[name]['frac_median']:.4f} "
              f"(best {res[name]['frac_best']:.4f})", flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
