#!/usr/bin/env python3
"""Diagnostic for test_batch_scope_scratch_mid_scope_flush_and_streams under GPU_MAX_HW_QUEUES=16: a scope
whose scratch partials (recorded on the default stream) are read by a perform_addition on another stream.
Prints, per trial, whether the rebuilt block and the written-out partial are right, and the flush stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "erasure-codes-prototype_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import ecg  # noqa: E402
from test_gpu_parity import _azure_repair_state, _repair_sequence  # noqa: E402


def main():
    torch.cuda.set_device(0)
    S, B = 8, 4096
    ec, st, plan = _azure_repair_state(ecg, torch, S, B, 0x5C2)
    ref_p = torch.zeros((S, 2, B), dtype=torch.uint8, device="cuda")
    ref_o = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
    _repair_sequence(ec, st, plan, ref_p, ref_o, B)
    torch.cuda.synchronize()
    for prio in (-1, 0):
        bad = 0
        for trial in range(20):
            partials = torch.full((S, 2, B), 0x3C, dtype=torch.uint8, device="cuda")
            out = torch.zeros((S, B), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            side = torch.cuda.Stream(priority=prio)
            with ecg.batch() as scope:
                scope.scratch(partials)
                for s, (e, surv, sets) in enumerate(plan):
                    for i in range(2):
                        ec.encode_partial_blocks_for_decoding([st[s, b] for b in sets[i]], [partials[s, i]], B,
                                                              sets[i], surv, [e])
                ec.perform_addition([partials[0, 0], partials[0, 1]], [out[0]], B, 2, 1, stream=side.cuda_stream)
            torch.cuda.synchronize()
            o = torch.equal(out[0], ref_o[0])
            p = torch.equal(partials[0], ref_p[0])
            bad += not (o and p)
            if not (o and p) or trial == 0:
                print(f"prio {prio} trial {trial}: out ok {o}, partial ok {p}, out==0x3C^0x3C {bool((out[0]==0).all())}, "
                      f"stats {ecg.batch_last_stats()}", flush=True)
        print(f"prio {prio}: {bad}/20 wrong", flush=True)


if __name__ == "__main__":
    main()
