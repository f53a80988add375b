"""Encode kernel time by HBM layout (RS(10,4), 1 MiB blocks, 4096 stripes), interleaved rounds in one
process.  Layouts:
  instripe   [S][14][B], parities written into the stripe (bench.py's layout; grid map 1 by the auto rule)
  separate   data [S][10][B] (the proxy's value buffer per stripe, proxy.cpp:337-339) + parities in their
             own [S][4][B] allocation (the proxy's separate coding buffers, proxy.cpp:335-342; map 2)
  blockmajor [14][S][B] in one allocation (block b of stripe s at b*S*B + s*B; parities a separate region)
Usage: python tools/layout_probe.py [--rounds R] [--maps 1,2]
"""
import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "erasure-codes-prototype_amd"))
import ecg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--maps", default="3")
    a = ap.parse_args()
    k, m, B, S = 10, 4, 1 << 20, a.stripes
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    inst = torch.empty((S, k + m, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(inst, 1)
    sep_d = inst[:, :k].clone()
    sep_p = torch.empty((S, m, B), dtype=torch.uint8, device="cuda")
    del inst
    torch.cuda.empty_cache()
    inst = torch.empty((S, k + m, B), dtype=torch.uint8, device="cuda")
    inst[:, :k].copy_(sep_d)
    layouts = {
        "instripe": (inst[:, :k], inst[:, k:]),
        "separate": (sep_d, sep_p),
    }
    bm = None
    if torch.cuda.mem_get_info()[0] > (k + m) * S * B + (4 << 30):
        bm = torch.empty((k + m, S, B), dtype=torch.uint8, device="cuda")
        bm[:k].copy_(sep_d.transpose(0, 1))
        layouts["blockmajor"] = (bm[:k].transpose(0, 1), bm[k:].transpose(0, 1))
    alg = S * (k + m) * B
    res = {name: [] for name in layouts}
    maps = [int(x) for x in a.maps.split(",")]
    for r in range(a.rounds):
        for gm in maps:
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, gm)
            for name, (d, p) in layouts.items():
                for _ in range(2):
                    ecg.encode_batch(k, m, M, d, p)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    ecg.encode_batch(k, m, M, d, p)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 3 / 1e3
                res[name].append((gm, t))
    ref = None
    for name, v in res.items():
        for gm in maps:
            ts = sorted(t for g, t in v if g == gm)
            med = ts[len(ts) // 2]
            print(f"{name:10s} map {gm}: median {med * 1e3:.3f} ms  min {ts[0] * 1e3:.3f} ms  "
                  f"{alg / med / 1e12:.3f} TB/s = {alg / med / 8e12:.3f} of 8 TB/s", flush=True)
    # parity bytes agree across layouts
    assert torch.equal(inst[:, k:], sep_p), "separate layout parities differ"
    if bm is not None:
        assert torch.equal(inst[:, k:], bm[k:].transpose(0, 1)), "block-major parities differ"
    print("parities identical across layouts")


if __name__ == "__main__":
    main()
