#!/usr/bin/env python3
"""Same encode, two kernel modes: the batched STRIDED launch (addresses from base + strides) against the
pointer-table PTRS launch (the deferred-batch scope's per-stripe calls on blocks that do not form one
strided batch), on one [S][k+m][B] batch.  Run under `rocprofv3 --kernel-trace --stats` (or --pmc) and
compare gf_vec_kernel<MT, 2, ...> (STRIDED) with gf_vec_kernel<MT, 1, ...> (PTRS).

The per-stripe calls are recorded in pair-swapped stripe order (1, 0, 3, 2, ...): the same blocks and
nearly the same DRAM order, but not one strided batch, so the flush takes the pointer-table launch.
--cols runs the PTRS launch at several ECG_OPT_COLS_PER_WG values (16-byte columns per workgroup).

    python profiles/r02/mode_probe/mode_probe.py [--block 1048576] [--stripes 4096] [--reps 5] [--cols 0,256,512]
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cols", default="0", help="comma-separated COLS_PER_WG values for the PTRS launch")
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
    order = [s ^ 1 for s in range(S)] if S % 2 == 0 else list(range(S))[::-1]
    data = [[st[s, j] for j in range(k)] for s in order]
    cod = [[st[s, k + i] for i in range(m)] for s in order]
    cols = [int(c) for c in a.cols.split(",")]
    saved = ecg.get_option(ecg.ECG_OPT_COLS_PER_WG)
    # The host records S per-stripe calls (tens of ms from Python) before a table launch; an idle GPU
    # drops its clocks in that gap (idle-gap effect), so a copy loop keeps it busy meanwhile and
    # the table launch and the strided launch run back to back behind it.
    fa = torch.empty(1 << 31, dtype=torch.uint8, device="cuda")
    fb = torch.empty_like(fa)
    for r in range(a.reps):
        for c in cols:  # kernel times: rocprofv3
            for strided_first in (False, True):  # both orders: the kernel right after the copies runs slower
                for _ in range(60):
                    fb.copy_(fa)
                if strided_first:
                    ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])
                ecg.set_option(ecg.ECG_OPT_COLS_PER_WG, c)
                with ecg.batch():
                    for s in range(S):
                        ec.encode(data[s], cod[s], B)
                ecg.set_option(ecg.ECG_OPT_COLS_PER_WG, saved)
                if not strided_first:
                    ecg.encode_batch(k, m, M, st[:, :k], st[:, k:])
                torch.cuda.synchronize()
        print(f"rep {r} done", flush=True)
    assert torch.equal(st, ref)
    print("outputs equal", flush=True)


if __name__ == "__main__":
    main()
