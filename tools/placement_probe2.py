#!/usr/bin/env python3
"""Placement probe, part 2: offsets INSIDE one allocation (tuning tool, one process, interleaved rounds).

tools/placement_probe.py showed the separate-output decode moving between 0.75 and 0.83 of HBM with the
output buffer it writes, and the encode between 0.77 and 0.79 with the stripe buffer, in one process.
Virtual-address offsets between separate allocations did not predict it, so this keeps everything in
ONE allocation per batch, where offsets are under the caller's control: X = [stripes | slack | outputs].
For two such allocations (X, Y) it times the encode with the stripes at byte offset 0 and 2 MiB, the
decode in place, and the separate-output decode with the outputs at the end of the stripes plus
d = 0, 1, 2, 3, 4, 6 MiB.  If the good and bad offsets agree between X and Y (and between processes),
the HBM address map is contiguous enough inside an allocation for a layout to pick the good one.
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
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, MiB, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    pats = [[e] for e in range(n)]
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    SB = S * n * B
    slack = 8 * MiB
    size = slack + SB + slack + S * B
    allocs = {name: torch.empty(size, dtype=torch.uint8, device="cuda") for name in ("X", "Y")}

    def stripes_at(buf, off):
        return buf[off:off + SB].view(S, n, B)

    def outputs_at(buf, d):
        o = slack + SB + d
        return buf[o:o + S * B].view(S, 1, B)

    variants = []
    for name, buf in allocs.items():
        for off in (0, 2 * MiB):
            st = stripes_at(buf, slack + off)
            ecg.fill_random(st, 0xEC0DE)
            variants.append((f"{name} encode stripes@{off // MiB}M",
                             (lambda st=st: ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])), S * n * B))
        st = stripes_at(buf, slack)
        ecg.fill_random(st, 0xEC0DE)
        ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])
        for d in (0, 1, 2, 3, 4, 6):
            out = outputs_at(buf, d * MiB)
            variants.append((f"{name} decode out@+{d}M", (lambda st=st, out=out: ecg.decode_batch(
                k, m, M, 1, pats, st, out=out, pattern_of_stripe=pos)), S * (k + 1) * B))
    print("allocations:", {kk: hex(v.data_ptr()) for kk, v in allocs.items()}, flush=True)
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
    out = {"allocations": {kk: hex(v.data_ptr()) for kk, v in allocs.items()}}
    for name, _, nbytes in variants:
        t = times[name]
        med = statistics.median(t)
        out[name] = {"median_ms": round(med, 3), "best_ms": round(min(t), 3),
                     "frac_median": round(nbytes / (med * 1e-3) / 8e12, 4)}
        print(f"{name:24s} median {med:7.3f} ms ({out[name]['frac_median']:.4f})", flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
