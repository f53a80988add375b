#!/usr/bin/env python3
"""Per-call latency of the host-buffer tier (the reference's own call pattern: one jerasure /
ErasureCode call per stripe on host memory, proxy.cpp:312-349).  Prints microseconds per call for the
config-1 shape (RS(6,4), 1 KiB) and a few larger blocks, for encode and single-erasure decode."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))

import numpy as np  # noqa: E402

import ecg  # noqa: E402


def per_call(fn, n):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--sweep-zc", action="store_true",
                    help="zero-copy threshold sweep: RS(10,4) 32-256 KiB blocks, DMA staging vs zero-copy")
    ap.add_argument("--sweep-lat", action="store_true",
                    help="latency-kernel lane width: RS(10,4) 1-256 KiB zero-copy calls, 4 vs 16 bytes per lane")
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    res = {}
    cases = [(zc, k, m, B) for zc in (0, 1 << 20) for k, m, B in
             [(6, 4, 1024), (10, 4, 1024), (10, 4, 16384), (10, 4, 65536), (10, 4, 1 << 20)]]
    if a.sweep_zc:
        cases = [(zc, 10, 4, B) for B in (32768, 65536, 98304, 131072, 196608, 262144) for zc in (0, 1 << 26)]
    lat = {}
    if a.sweep_lat:  # zc slot carries the ECG_OPT_LAT_DWORD_BYTES value; zero-copy stays at its default
        cases = [(lw, 10, 4, B) for r in range(2) for B in (1024, 4096, 16384, 32768, 65536, 131072, 262144)
                 for lw in (0, 1 << 20)]
    for zc, k, m, B in cases:
        if a.sweep_lat:
            ecg.set_option(ecg.ECG_OPT_LAT_DWORD_BYTES, zc)
        else:
            ecg.set_option(ecg.ECG_OPT_ZEROCOPY_BYTES, zc)
        M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
        data = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(k)]
        coding = [np.zeros(B, np.uint8) for _ in range(m)]
        n = a.calls if B <= 65536 else max(50, a.calls // 20)
        enc = per_call(lambda: ecg.jerasure_matrix_encode(k, m, M, data, coding, B), n)
        er = [3, -1]
        dec = per_call(lambda: ecg.jerasure_matrix_decode(k, m, M, 1, er, data, coding, B), n)
        name = f"RS({k},{m}) B={B} " + (f"lat_dword<={zc}" if a.sweep_lat else f"zerocopy<={zc}")
        if name in res:
            name += " (round 2)"
        res[name] = {"encode_us": round(enc, 1), "decode_us": round(dec, 1),
                     "encode_GBps_data": round(k * B / enc / 1e3, 3)}
        print(f"{name:40s} encode {enc:9.1f} us/call   decode {dec:9.1f} us/call", flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
