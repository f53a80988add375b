"""Occupancy A/B in one process on the same buffers: the headline step (RS(10,4) 1 MiB x 4096: encode, then
the rotating 1-erasure decode into the arena's rebuild blocks, as bench.py lays it out) run through each
libecg variant in rotation (ABBA over ROUNDS rounds).  libecg_ldsN.so launches every kernel with N bytes
of unused dynamic LDS (build_lds_variants.sh): at most floor(160 KiB / N) workgroups per CU.  Every
variant's parities and rebuilt blocks are compared with the product library's.
usage: python occ_probe.py ROUNDS lib1[:OPT=V,...] lib2 ...   (paths relative to erasure-codes-prototype_amd/lib;
options set in that library only)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
import ecg  # noqa: E402
import torch  # noqa: E402

rounds, names = int(sys.argv[1]), sys.argv[2:]
libdir = os.path.join(ROOT, "erasure-codes-prototype_amd", "lib")
libs = {}
for n in names:  # "lib.so" or "lib.so:OPT=V,OPT=V" (ECG_OPT_* set in that library only)
    path, _, opts = n.partition(":")
    ecg.LIB_PATH, ecg._L = os.path.join(libdir, path), None
    libs[n] = ecg.lib()
    for kv in filter(None, opts.split(",")):
        o, v = kv.split("=")
        ecg.set_option(int(o), int(v))
k, m, B, S = 10, 4, 1 << 20, 4096
n_ = k + m
M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
patterns = [[e] for e in range(n_)]
arena = torch.empty(S * (n_ + 1) * B, dtype=torch.uint8, device="cuda")
stripes = arena[:S * n_ * B].view(S, n_, B)
rebuilt = arena[S * n_ * B:].view(S, 1, B)
ecg.fill_random(stripes, 0xEC0DE)
pos = (torch.arange(S, device="cuda", dtype=torch.int32) % n_).contiguous()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
times = {n: {"encode": [], "decode": []} for n in names}
ref = None
for r in range(rounds):
    for n in (names if r % 2 == 0 else names[::-1]):
        ecg._L = libs[n]
        for rep in range(3):  # two warm steps, then the timed one
            ev[0].record()
            ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])
            ev[1].record()
            ecg.decode_batch(k, m, M, 1, patterns, stripes, out=rebuilt, pattern_of_stripe=pos)
            ev[2].record()
        ev[2].synchronize()
        times[n]["encode"].append(ev[0].elapsed_time(ev[1]))
        times[n]["decode"].append(ev[1].elapsed_time(ev[2]))
        if r == 0:
            cs = (int(stripes[:, k:].view(torch.int64).sum().item()), int(rebuilt.view(torch.int64).sum().item()))
            ref = ref or cs
            assert cs == ref, (n, "outputs differ from the first library's")
out = {}
for n, t in times.items():
    e, d = t["encode"], t["decode"]
    out[n] = {"encode_frac_mean": round(S * 14 * B / (sum(e) / len(e) / 1e3) / 8e12, 4),
              "encode_frac_best": round(S * 14 * B / (min(e) / 1e3) / 8e12, 4),
              "decode_frac_mean": round(S * 11 * B / (sum(d) / len(d) / 1e3) / 8e12, 4),
              "decode_frac_best": round(S * 11 * B / (min(d) / 1e3) / 8e12, 4), "n": len(e)}
print(json.dumps(out))
