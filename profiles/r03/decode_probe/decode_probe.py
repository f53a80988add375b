#!/usr/bin/env python3
"""Config-2 decode leg, output placement x grid map (tuning tool, one process, interleaved rounds).

bench.py's decode writes the rebuilt block of every stripe into a separate [S][1][B] buffer; the
reference's jerasure_matrix_decode writes it in place, into the erased block of the stripe itself
(rs.cpp:36, erasures are outputs).  Both move (k + 1) * B per stripe.  Variants, each timed by HIP events
over `reps` launches per round, rounds interleaved: separate output / in place, with the auto grid map and
with map 1 / map 2 forced.  Prints the median and best launch time and the algorithmic HBM fraction.
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, a.block, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 0xEC0DE)
    ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])
    ref = stripes.view(torch.int64).sum().item()
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    pats = [[e] for e in range(n)]
    saved = ecg.get_option(ecg.ECG_OPT_GRID_MAP)

    def run(inplace, gm):
        ecg.set_option(ecg.ECG_OPT_GRID_MAP, gm)
        ecg.decode_batch(k, m, M, 1, pats, stripes, out=None if inplace else rebuilt, pattern_of_stripe=pos)

    variants = {"separate auto(2)": (False, 3), "separate map1": (False, 1), "inplace auto(1)": (True, 3),
                "inplace map2": (True, 2)}
    times = {v: [] for v in variants}
    for _ in range(2):  # warm-up
        for v, (ip, gm) in variants.items():
            run(ip, gm)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for v, (ip, gm) in variants.items():
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            evs[0].record()
            for i in range(a.reps):
                run(ip, gm)
                evs[i + 1].record()
            torch.cuda.synchronize()
            times[v] += [evs[i].elapsed_time(evs[i + 1]) for i in range(a.reps)]
    ecg.set_option(ecg.ECG_OPT_GRID_MAP, saved)
    assert stripes.view(torch.int64).sum().item() == ref, "in-place decode changed the stripes"
    idx = torch.arange(S, device="cuda")
    assert torch.equal(rebuilt[:, 0], stripes[idx, idx % n])
    alg = S * (k + 1) * B
    res = {}
    for v, t in times.items():
        med, best = statistics.median(t), min(t)
        res[v] = {"median_ms": round(med, 3), "best_ms": round(best, 3),
                  "frac_median": round(alg / (med * 1e-3) / 8e12, 4), "frac_best": round(alg / (best * 1e-3) / 8e12, 4)}
        print(f"{v:18s} median {med:7.3f} ms ({res[v]['frac_median']:.4f})  best {best:7.3f} ms ({res[v]['frac_best']:.4f})")
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
