#!/usr/bin/env python3
"""Does a kernel's rate depend on what ran before it?  The bench's decode (after an encode) measures
0.76 of 8 TB/s while the microbench's decode (after a decode) measures 0.81.  This times the default
config-2 encode and decode kernels in several orders within one process, HIP events around each.

    python profiles/r01/order_probe.py [--reps 6]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
import torch  # noqa: E402

import ecg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--pattern", action="store_true", help="measurement patterns instead of orders (no idle)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, 1 << 20, 4096
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 1)
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    pats = [[e] for e in range(n)]
    data, coding = stripes[:, :k], stripes[:, k:]
    enc_b, dec_b = S * n * B, S * (k + 1) * B

    def enc():
        ecg.encode_batch(k, m, M, data, coding)

    def dec():
        ecg.decode_batch(k, m, M, 1, pats, stripes, out=rebuilt, pattern_of_stripe=pos)

    def idle():
        torch.cuda.synchronize()
        time.sleep(0.05)

    # each sequence: list of (name, fn, bytes or None); timed entries get events
    seqs = {
        "enc;dec (bench order)": [("enc", enc, enc_b), ("dec", dec, dec_b)],
        "dec;dec": [("dec0", dec, dec_b), ("dec", dec, dec_b)],
        "enc;enc": [("enc0", enc, enc_b), ("enc", enc, enc_b)],
        "dec;enc": [("dec", dec, dec_b), ("enc", enc, enc_b)],
        "idle 50 ms;dec": [("idle", idle, None), ("dec", dec, dec_b)],
        "idle 50 ms;enc": [("idle", idle, None), ("enc", enc, enc_b)],
    }
    enc()
    dec()
    torch.cuda.synchronize()
    if a.pattern:
        pattern_probe(enc, dec, enc_b, dec_b, a.reps)
        # the microbench copies the first half of the stripe batch over the second half before its later
        # decode rounds: does the data (not the access pattern) change the rate?
        flat = stripes.view(S * n, B)
        half = S * n // 2
        flat[half:2 * half].copy_(flat[:half])
        torch.cuda.synchronize()
        print("-- after copying the first half of the batch over the second half", flush=True)
        pattern_probe(enc, dec, enc_b, dec_b, a.reps)
        ecg.fill_random(stripes, 1)
        rebuilt.zero_()
        torch.cuda.synchronize()
        print("-- refilled with random bytes, rebuilt zeroed", flush=True)
        pattern_probe(enc, dec, enc_b, dec_b, a.reps)
        return
    res = {}
    for _ in range(a.reps):
        for sname, seq in seqs.items():
            evs = []
            for name, fn, nb in seq:
                if nb is None:
                    fn()
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                evs.append((name, nb, e0, e1))
            torch.cuda.synchronize()
            for name, nb, e0, e1 in evs:
                res.setdefault((sname, name), []).append(nb / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    for (sname, name), v in res.items():
        print(f"{sname:24s} {name:5s} median {statistics.median(v):7.1f} GB/s ({statistics.median(v) / 8000:.3f})  "
              f"min {min(v):7.1f}  max {max(v):7.1f}", flush=True)


def pattern_probe(enc, dec, enc_b, dec_b, reps):
    """Same kernels, different measurement patterns, no idle periods: microbench-style (warm call, sync,
    R back-to-back calls each between two events) vs bench-style (enc, dec alternating, 3 events per step)."""
    def ev():
        return torch.cuda.Event(enable_timing=True)

    def rate(nb, a, b):
        return nb / (a.elapsed_time(b) * 1e-3) / 1e9

    for rnd in range(2):
        for name, fn, nb in (("dec", dec, dec_b), ("enc", enc, enc_b)):
            fn()
            torch.cuda.synchronize()
            evs = [(ev(), ev()) for _ in range(reps)]
            for a0, a1 in evs:
                a0.record()
                fn()
                a1.record()
            torch.cuda.synchronize()
            v = [rate(nb, a0, a1) for a0, a1 in evs]
            print(f"round {rnd} back-to-back {name}: median {statistics.median(v):7.1f} GB/s "
                  f"({statistics.median(v) / 8000:.3f})", flush=True)
        evs = [(ev(), ev(), ev()) for _ in range(reps)]
        for e0, e1, e2 in evs:
            e0.record()
            enc()
            e1.record()
            dec()
            e2.record()
        torch.cuda.synchronize()
        ve = [rate(enc_b, e0, e1) for e0, e1, _ in evs]
        vd = [rate(dec_b, e1, e2) for _, e1, e2 in evs]
        print(f"round {rnd} bench-style   enc: median {statistics.median(ve):7.1f} ({statistics.median(ve) / 8000:.3f})"
              f"  dec: median {statistics.median(vd):7.1f} ({statistics.median(vd) / 8000:.3f})", flush=True)


if __name__ == "__main__":
    main()
