"""Config 5's block size (RS(10,4), 4 MiB) against the headline's (1 MiB) on the encode, in one process on
the same buffers: one 1024-stripe wave at 4 MiB (config 5's wave) and the 4096-stripe 1 MiB batch (the
headline), each encoded under several launch settings in rotation (grid map, chunk size), ROUNDS rounds.
Prints per (shape, setting) the mean / best fraction of 8 TB/s for the algorithmic bytes.  Speed only: the
parities of every setting are compared with the first setting's.
usage: python b4m_probe.py [ROUNDS]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
import ecg  # noqa: E402
import torch  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
k, m = 10, 4
M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
SETTINGS = [("auto", {}), ("map2", {ecg.ECG_OPT_GRID_MAP: 2}), ("map0", {ecg.ECG_OPT_GRID_MAP: 0}),
            ("chunk4k", {ecg.ECG_OPT_COLS_PER_WG: 256}), ("chunk8k", {ecg.ECG_OPT_COLS_PER_WG: 512})]
shapes = {"4MiB_x1024": (1024, 4 << 20), "1MiB_x4096": (4096, 1 << 20)}
bufs = {}
for name, (S, B) in shapes.items():
    t = torch.empty((S, k + m, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(t, 0xEC0DE)
    bufs[name] = t
saved = {o: ecg.get_option(o) for o in (ecg.ECG_OPT_GRID_MAP, ecg.ECG_OPT_COLS_PER_WG)}
times = {(n, s): [] for n in shapes for s, _ in SETTINGS}
ref = {}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for r in range(rounds):
    order = SETTINGS if r % 2 == 0 else SETTINGS[::-1]
    for name, (S, B) in shapes.items():
        buf = bufs[name]
        for sname, opts in order:
            for o, v in saved.items():
                ecg.set_option(o, v)
            for o, v in opts.items():
                ecg.set_option(o, v)
            ecg.encode_batch(k, m, M, buf[:, :k], buf[:, k:])  # warm this setting
            torch.cuda.synchronize()
            ev[0].record()
            ecg.encode_batch(k, m, M, buf[:, :k], buf[:, k:])
            ev[1].record()
            ev[1].synchronize()
            times[(name, sname)].append(ev[0].elapsed_time(ev[1]))
            if r == 0:
                cs = int(buf[:, k:].view(torch.int64).sum().item())
                ref.setdefault(name, cs)
                assert cs == ref[name], (name, sname, "parities differ between settings")
for o, v in saved.items():
    ecg.set_option(o, v)
out = {}
for (name, sname), v in times.items():
    S, B = shapes[name]
    alg = S * (k + m) * B
    out.setdefault(name, {})[sname] = {"mean_ms": round(sum(v) / len(v), 3), "frac_mean": round(alg / (sum(v) / len(v) / 1e3) / 8e12, 4),
                                      "frac_best": round(alg / (min(v) / 1e3) / 8e12, 4), "n": len(v)}
print(json.dumps(out))
