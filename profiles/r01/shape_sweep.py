#!/usr/bin/env python3
"""Grid-map sweep over program shapes (tuning only): k_in inputs -> m_out outputs per stripe, outputs
written either inside the stripe (encode-like) or to a separate compact buffer (decode-like), for each
grid map.  One process, interleaved rounds, HIP-event timing; prints algorithmic GB/s."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ecg  # noqa: E402
from microbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--maps", default="1,2")
    ap.add_argument("--out", default=None)
    ap.add_argument("--shapes", default="grid", choices=["grid", "baseline"],
                    help="grid: k_in x m_out in {1,4,10} x {1,2,4}; baseline: the shapes the BASELINE workloads run")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    S, B, n = a.stripes, a.block, 14
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 7)
    sep = torch.empty((S, 4, B), dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(1)
    variants = []
    if a.shapes == "grid":
        shapes = [(k, mm, w) for k in (1, 4, 10) for mm in (1, 2, 4) for w in ("in-stripe", "separate")]
    else:  # RS(10,4) encode / decodes, Azure(12,2,2) encode + local/global repair, PC row merge, partials
        shapes = [(10, 4, "in-stripe"), (10, 1, "separate"), (10, 2, "separate"), (10, 4, "separate"),
                  (12, 2, "in-stripe"), (6, 1, "separate"), (12, 1, "separate"), (8, 1, "separate"),
                  (3, 1, "separate"), (4, 1, "separate")]
    for k_in, m_out, where_only in shapes:
        if True:
            coef = rng.integers(2, 256, size=(m_out, k_in))
            src = list(range(k_in))
            for where in (where_only,):
                if where == "in-stripe":
                    dst, out = list(range(k_in, k_in + m_out)), stripes
                else:
                    dst, out = list(range(m_out)), sep
                for gmap in [int(x) for x in a.maps.split(",")]:
                    name = f"k={k_in:2d} m={m_out} {where:9s} map={gmap}"
                    fn = (lambda c=coef, s=src, d=dst, o=out: ecg.matrix_apply_batch(c, s, d, stripes, o))
                    variants.append((name, gmap, fn, S * (k_in + m_out) * B))
    res = {v[0]: [] for v in variants}
    for _ in range(a.rounds):
        for name, gmap, fn, nbytes in variants:
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, gmap)
            res[name] += [nbytes / (t * 1e-3) / 1e9 for t in timeit(fn, a.reps)]
    ecg.set_option(ecg.ECG_OPT_GRID_MAP, 1)
    out = {}
    for name, *_ in variants:
        med = statistics.median(res[name])
        out[name] = round(med, 1)
        print(f"{name:36s} {med:8.1f} GB/s ({med / 8000 * 100:5.1f}%)", flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
