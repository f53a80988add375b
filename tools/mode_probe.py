#!/usr/bin/env python3
"""Same encode, two kernel modes: the batched STRIDED launch (addresses from base + strides) against
the pointer-table PTRS launch (the deferred-batch scope's per-stripe calls), on one [S][k+m][B] batch.
Run under `rocprofv3 --kernel-trace --stats` and compare gf_vec_kernel<MT, 2, ...> (STRIDED) with
gf_vec_kernel<MT, 1, ...> (PTRS); the script also prints event-timed rates of the STRIDED launch.

    python tools/mode_probe.py [--block 1048576] [--stripes 4096] [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd")]
import torch  # noqa: E402

import ecg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k, m, B, S = 10, 4, a.block, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    st = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(st, 3)
    ref = st.clone()
    ecg.encode_batch(k, m, M, ref[:, :k], ref[:, k:])
    ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=k, m=m))
    data = [[st[s, j] for j in range(k)] for s in range(S)]
    cod = [[st[s, k + i] for i in range(m)] for s in range(S)]
    for r in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])
        e1.record()
        torch.cuda.synchronize()
        print(f"STRIDED rep {r}: {S * n * B / (e0.elapsed_time(e1) * 1e-3) / 8e12:.3f} of 8 TB/s", flush=True)
        with ecg.batch():
            for s in range(S):
                ec.encode(data[s], cod[s], B)
        torch.cuda.synchronize()
    assert torch.equal(st, ref)
    print("outputs equal", flush=True)


if __name__ == "__main__":
    main()
