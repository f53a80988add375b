import sys, os
ROOT = os.path.join(os.path.dirname(__file__), "..", "..", "..")
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import ecg
import bench
torch.cuda.set_device(0)
for name, t, params, _ in bench.FAMILIES:
    cp = ecg.CodingParameters(**params)
    h = ecg.ec_factory(t, cp)
    h.init_coding_parameters(cp)
    k, m = h.k, h.m
    n = k + m
    bad = []
    for i in range(n):
        pat = sorted({i, (i + n // 2) % n})
        st = [np.zeros(64, np.uint8) for _ in range(n)]
        st[(pat[-1] + 1) % n][:] = 5
        rc = h.decode(st[:k], st[k:], 64, pat + [-1], len(pat))
        if rc:
            bad.append((pat, rc))
    M = h.make_encoding_matrix() if t < 7 else None
    print(name, k, m, "bad:", bad[:4], "M rows" if M else "", flush=True)
