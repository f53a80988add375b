#!/usr/bin/env python3
"""Config-2 decode leg: runtime knobs swept together (tuning tool, one process, interleaved rounds).

The separate-output decode (bench.py's decode leg) is the half of the headline that moves most between
boxes (0.760-0.817 across the driver's and the builder's runs, encode 0.78-0.79 on the same boxes).
tools/decode_probe.py covered output placement x grid map; this sweeps the rest of the runtime knobs on
the same launch: non-temporal policy (ECG_OPT_NT), columns per workgroup (ECG_OPT_COLS_PER_WG) and the
stripe run length of grid map 2 (ECG_OPT_MAP_GROUP), with the encode at its defaults and at each NT
policy as the box's reference.  Each variant: `reps` HIP-event-timed launches per round, rounds
interleaved; prints median / best launch time and the algorithmic HBM fraction ((k + 1) B S per decode,
(k + m) B S per encode, / 8 TB/s).
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
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    pats = [[e] for e in range(n)]
    knobs = (ecg.ECG_OPT_NT, ecg.ECG_OPT_COLS_PER_WG, ecg.ECG_OPT_GRID_MAP, ecg.ECG_OPT_MAP_GROUP)
    saved = [ecg.get_option(o) for o in knobs]

    def dec():
        ecg.decode_batch(k, m, M, 1, pats, stripes, out=rebuilt, pattern_of_stripe=pos)

    def enc():
        ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])

    dec_bytes, enc_bytes = S * (k + 1) * B, S * n * B
    variants = []  # (name, fn, bytes, {option: value})
    variants.append(("decode defaults", dec, dec_bytes, {}))
    variants.append(("encode defaults", enc, enc_bytes, {}))
    for nt in (0, 1, 2):
        variants.append((f"decode nt={nt}", dec, dec_bytes, {ecg.ECG_OPT_NT: nt}))
        variants.append((f"encode nt={nt}", enc, enc_bytes, {ecg.ECG_OPT_NT: nt}))
    for cpw in (256, 512):
        variants.append((f"decode cpw={cpw}", dec, dec_bytes, {ecg.ECG_OPT_COLS_PER_WG: cpw}))
    for g in (2, 4, 8, 16):
        variants.append((f"decode map2 G={g}", dec, dec_bytes, {ecg.ECG_OPT_GRID_MAP: 2, ecg.ECG_OPT_MAP_GROUP: g}))
    variants.append(("decode map1", dec, dec_bytes, {ecg.ECG_OPT_GRID_MAP: 1}))
    variants.append(("decode nt=1 cpw=256", dec, dec_bytes, {ecg.ECG_OPT_NT: 1, ecg.ECG_OPT_COLS_PER_WG: 256}))

    def setup(opts):
        for o, v in zip(knobs, saved):
            ecg.set_option(o, opts.get(o, v))

    times = {v[0]: [] for v in variants}
    for _ in range(2):  # warm-up
        for name, fn, _, opts in variants:
            setup(opts)
            fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, fn, _, opts in variants:
            setup(opts)
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            evs[0].record()
            for i in range(a.reps):
                fn()
                evs[i + 1].record()
            torch.cuda.synchronize()
            times[name] += [evs[i].elapsed_time(evs[i + 1]) for i in range(a.reps)]
    setup({})
    out = {}
    for name, _, nbytes, _ in variants:
        t = times[name]
        med, best = statistics.median(t), min(t)
        out[name] = {"median_ms": round(med, 3), "best_ms": round(best, 3),
                     "frac_median": round(nbytes / (med * 1e-3) / 8e12, 4),
                     "frac_best": round(nbytes / (best * 1e-3) / 8e12, 4)}
        print(f"{name:24s} median {med:7.3f} ms ({out[name]['frac_median']:.4f})  best {best:7.3f} ms "
              f"({out[name]['frac_best']:.4f})", flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
