import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "..", "erasure-codes-prototype_amd"))
import numpy as np
import torch
import ecg
torch.cuda.set_device(0)
for B in (64, 1024, 4096):
    for fresh in (True, False):
        h = ecg.ec_factory(0, ecg.CodingParameters(k=12, m=4))
        if not fresh:
            h.init_coding_parameters(ecg.CodingParameters(k=12, m=4))
            h.generate_partition()
            h.generate_repair_plan([0])
        st = [np.zeros(B, np.uint8) for _ in range(16)]
        st[1][:] = 7
        er = [0, 8, -1]
        rc = h.decode(st[:12], st[12:], B, er, 2)
        print(B, fresh, rc, ecg.lib().ecg_last_error(), st[0][:4], st[8][:4], flush=True)
