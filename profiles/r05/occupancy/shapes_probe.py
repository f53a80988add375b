"""ECG_OPT_MT1_LDS_PAD over single-output shapes, inside one process on the same buffers: for k inputs
(BINARY all-ones row, or a GENERAL row) one strided batch launch k -> 1 over [S][k][1 MiB] into a
separate [S][1][1 MiB] output (decode / repair / merge layout), about 44 GiB per shape; every pad value in
rotation (forward / backward on alternate rounds), ROUNDS rounds; per (shape, pad) the mean fraction of
8 TB/s for the algorithmic bytes.  Outputs are compared across pads.
usage: python shapes_probe.py ROUNDS K1,K2,... PAD1 PAD2 ...   (ECG_PROBE_M=m: k -> m launches instead)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
import ecg  # noqa: E402
import torch  # noqa: E402

rounds, ks, pads = int(sys.argv[1]), [int(x) for x in sys.argv[2].split(",")], [int(x) for x in sys.argv[3:]]
M_OUT = int(os.environ.get("ECG_PROBE_M", "1"))
B = 1 << 20
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
saved = ecg.get_option(ecg.ECG_OPT_MT1_LDS_PAD)
out = {}
try:
    for k in ks:
        S = (44 << 30) // ((k + M_OUT) * B) // 64 * 64
        d_in = torch.empty((S, k, B), dtype=torch.uint8, device="cuda")
        d_out = torch.empty((S, M_OUT, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(d_in, 0xEC0DE + k)
        for flavour, row in (("binary", [1] * (k * M_OUT)),
                             ("general", [(7 * j + 3 + 31 * p) % 255 + 1 for p in range(M_OUT) for j in range(k)])):
            times = {p: [] for p in pads}
            ref = None
            for r in range(rounds):
                for p in (pads if r % 2 == 0 else pads[::-1]):
                    ecg.set_option(ecg.ECG_OPT_MT1_LDS_PAD, p)
                    ecg.matrix_apply_batch(row, list(range(k)), list(range(M_OUT)), d_in, d_out)  # warm
                    ev[0].record()
                    ecg.matrix_apply_batch(row, list(range(k)), list(range(M_OUT)), d_in, d_out)
                    ev[1].record()
                    ev[1].synchronize()
                    times[p].append(ev[0].elapsed_time(ev[1]))
                    if r == 0:
                        cs = int(d_out.view(torch.int64).sum().item())
                        ref = ref if ref is not None else cs
                        assert cs == ref, (k, flavour, p, "output differs between pads")
            alg = S * (k + M_OUT) * B
            key = f"{k}->{M_OUT} {flavour}"
            out[key] = {str(p): round(alg / (sum(v) / len(v) / 1e3) / 8e12, 4) for p, v in times.items()}
            print(key, out[key], flush=True)
        del d_in, d_out
        torch.cuda.empty_cache()
finally:
    ecg.set_option(ecg.ECG_OPT_MT1_LDS_PAD, saved)
print(json.dumps(out))
