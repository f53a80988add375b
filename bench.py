#!/usr/bin/env python3
"""bench.py — BASELINE.json's headline metric on MI355X.

Metric: "GiB/s encode + single-block decode (device-resident), RS(10,4) 1 MiB blocks, 1 & 8 GPU".
Workload (BASELINE.json configs[1]): RS(k=10, m=4), block_size = 1 MiB, a batch of S = 4096 stripes
per GPU resident in HBM ([S][14][1 MiB] = 56 GiB + a 4 GiB rebuild buffer).  One step = one pass of
the hot path over the batch:
  1. encode:  jerasure_matrix_encode of every stripe   (ecg_encode_batch, one launch)
  2. decode:  every stripe loses block e = s mod 14 and rebuilds it with jerasure_matrix_decode
              semantics (row_k_ones = failed_num, rs.cpp:36) into the rebuild buffer
              (ecg_decode_batch, 14 composed patterns, one launch)
value = data bytes coded per second over all ranks = N * S * 2 * k * B / t_max  (GiB/s; each pass
reads k data-sized blocks per stripe).  Inputs are synthetic splitmix64 bytes generated on the GPU
before the timed region.

Multi-GPU: stripes are independent, so each rank runs its own S stripes (weak scaling, no data-path
collective); one barrier + synchronize brackets the timed region, the elapsed time is max-reduced.

Extra JSON fields: roofline (dominant kernel = the encode kernel, timed with HIP events on the
stream it runs on; algorithmic bytes = (k+m)*B per stripe), cpu_baseline (oracle CPU restatement of
the same step on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ecg  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU (BASELINE configs[1]: 4096)")
    ap.add_argument("--block-size", type=int, default=1 << 20)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    return ap.parse_args()


def cpu_baseline(k, m, B, target_s):
    """Oracle CPU restatement (Jerasure algorithm, SIMD split tables) of the same step on a bounded
    sample: encode + single-erasure decode of S_cpu stripes, one jerasure call per stripe, threads =
    min(16, cpu_count)."""
    import numpy as np
    from oracle import ref
    ref.build()
    threads = max(1, min(16, os.cpu_count() or 1))
    S = 4 * threads
    M = ref.reed_sol_vandermonde_coding_matrix(k, m)
    n = k + m
    stripes = np.zeros((S, n, B), np.uint8)
    stripes[:, :k] = ref.splitmix_bytes(0xEC0DE, 0, S * k * B).reshape(S, k, B)
    data = np.ascontiguousarray(stripes[:, :k])
    coding = np.zeros((S, m, B), np.uint8)
    out = np.zeros((S, B), np.uint8)
    reps, t_total = 0, 0.0
    while t_total < target_s and reps < 1000:
        t0 = time.perf_counter()
        ref.encode_batch_mt(k, m, M, data, coding, B, S, threads)
        t1 = time.perf_counter()
        stripes[:, k:] = coding
        t2 = time.perf_counter()
        ref.decode_batch_mt(k, m, M, stripes, out, B, S, threads)
        t3 = time.perf_counter()
        t_total += (t1 - t0) + (t3 - t2)
        reps += 1
    gib = reps * S * 2 * k * B / 2 ** 30
    return {"value": round(gib / t_total, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x (encode + 1-erasure decode) of {S} RS({k},{m}) stripes x {B} B, "
                      f"one jerasure call per stripe, {threads} host threads, {t_total:.1f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    ecg.lib().ecg_set_device(torch.cuda.current_device())
    k, m, B, S = a.k, a.m, a.block_size, a.stripes
    n = k + m
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)

    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 0xEC0DE, word_offset=rank * (S * n * B // 8))
    pattern_of_stripe = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    patterns = [[e] for e in range(n)]
    data, coding = stripes[:, :k], stripes[:, k:]

    # HIP events on torch's current stream, which is the stream ecg launches on (ecg._stream)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]

    def step(ev=None):
        if ev:
            ev[0].record()
        ecg.encode_batch(k, m, M, data, coding)
        if ev:
            ev[1].record()
        ecg.decode_batch(k, m, M, 1, patterns, stripes, out=rebuilt, pattern_of_stripe=pattern_of_stripe)
        if ev:
            ev[2].record()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # sanity: the rebuilt blocks equal the erased originals (checked once, outside the timed region)
    idx = torch.arange(S, device="cuda")
    assert torch.equal(rebuilt[:, 0], stripes[idx, idx % n]), "decode mismatch"

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    enc_ms = [e[0].elapsed_time(e[1]) for e in evs]
    dec_ms = [e[1].elapsed_time(e[2]) for e in evs]
    step_bytes = S * 2 * k * B  # data read by encode + data read by decode
    value = world * step_bytes * a.steps / elapsed / 2 ** 30
    enc_avg = sum(enc_ms) / len(enc_ms) / 1e3
    dec_avg = sum(dec_ms) / len(dec_ms) / 1e3
    enc_bytes = S * (k + m) * B          # algorithmic HBM bytes of one encode launch
    dec_bytes = S * (k + 1) * B          # one decode launch
    achieved = enc_bytes / enc_avg / 1e9
    traffic = None
    if os.path.exists(PMC_FILE):
        try:
            pm = json.load(open(PMC_FILE))
            if pm.get("workload") == f"rs{k}{m}_B{B}_S{S}":
                traffic = pm.get("encode_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        line = {
            "metric": "GiB/s encode + single-block decode (device-resident), RS(10,4) 1 MiB blocks, 1 & 8 GPU",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)",
            "config": {"workload": f"RS({k},{m}) encode + rotating 1-erasure decode (e = s mod {n})",
                       "block_size": B, "stripes_per_gpu": S, "global_stripes": S * world,
                       "parallelism": f"stripes sharded over {world} GPU(s), no data-path collective"},
            "encode_gibps_per_gpu": round(S * k * B / enc_avg / 2 ** 30, 2),
            "decode_gibps_per_gpu": round(S * k * B / dec_avg / 2 ** 30, 2),
            "encode_ms": round(enc_avg * 1e3, 3),
            "decode_ms": round(dec_avg * 1e3, 3),
            "roofline": {"bound": "hbm", "kernel": "gf_vec_kernel<MT=4,STRIDED> (encode)",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "algorithmic_bytes_per_launch": enc_bytes,
                         "decode_achieved": round(dec_bytes / dec_avg / 1e9, 1)},
        }
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(k, m, B, a.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
