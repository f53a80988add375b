#!/usr/bin/env python3
"""bench.py — BASELINE.json's headline metric on MI355X (plus the other BASELINE configs on request).

Default workload (BASELINE.json configs[1], what the driver runs):
  RS(k=10, m=4), block_size = 1 MiB, S = 4096 stripes per GPU resident in HBM ([S][14][1 MiB] = 56 GiB
  + a 4 GiB rebuild buffer).  One step = one pass of the hot path over the batch:
    1. encode: jerasure_matrix_encode of every stripe                         (ecg_encode_batch)
    2. decode: stripe s loses block e = s mod 14 and rebuilds it with jerasure_matrix_decode semantics
       (row_k_ones = failed_num, rs.cpp:36) into the rebuild buffer  (ecg_decode_batch, 14 patterns)
  value = N * S * 2 * k * B / t_max in GiB/s (each pass reads k data-sized blocks per stripe).
  Inputs: splitmix64 bytes generated on the GPU before the timed region.
  The same line also carries, after the headline's buffers are freed:
    per_rank  every rank's encode / decode kernel time and HBM fraction (all-gathered);
    config5   BASELINE.json configs[4] at this N: RS(10,4), 4 MiB, 65536 stripes sharded over the ranks
              in HBM-resident waves of 1024 -- aggregate GiB/s, every rank's HBM fraction, and the
              combined parity checksum against the N = 1 value (--no-config5 skips it);
    host_path RS(10,4) 1 MiB stripes in pinned host memory, encode and 1-erasure decode including the
              PCIe copies (128 stripes per rank, every rank on its own link; --no-host-path skips it);
    ring_repair  config 3's partial decoding across neighbouring GPUs, partials over RCCL point to point
              (the lrc-repair-ring workload, 1024 repairs per rank; --no-ring skips it and the next); at
              N = 1 the rank is its own RCCL peer, so the same RCCL path runs on one GPU (an on-GPU copy);
    global_ring_repair  the same for global-parity repairs, four helper partitions on ranks q+1..q+4
              (lrc-global-ring, 256 repairs per rank, four partials each);
    merge_ring  configs[3]'s stripe merging with the old stripes' clusters on neighbouring GPUs
              (pc-merge-ring, 64 merges per rank, five 4 MiB row partials each).

Other workloads (--workload; measured for DESIGN.md, not the driver's BENCH line):
  lrc-repair  configs[2]: Azure-LRC(12,2,2), 1 MiB, single-block repair of block s mod 16 of every
              stripe, partial_decoding=true (helper partials + main partial + perform_addition) and the
              fused single-launch form;
  lrc-repair-ring  configs[2]'s partial decoding with helper and main proxies on neighbouring GPUs:
              helper partials sent over xGMI (RCCL point to point), added in the main rank's fused kernel;
  pc-merge    configs[3]: PC(4,1,4,1), 4 MiB blocks, stripe merging x=2 (HORIZONTAL): the 5 row
              parities of the merged PC(8,1,4,1) recomputed from the two old stripes;
  rs4m-waves  configs[4]: RS(10,4), 4 MiB blocks, 65536 stripes split over the ranks, encoded in
              HBM-resident waves of 1024 stripes (input regenerated per wave outside the timing);
  rs-host     configs[1] with the blocks in pinned HOST memory: the rate including hipMemcpyAsync to and
              from the GPU over PCIe (H2D -> kernel -> D2H pipeline), for DESIGN.md;
  rs-small-host  configs[0]'s shape: RS(6,4), 1 KiB blocks, one jerasure_matrix_encode per stripe on
              host buffers, issued from C++ (loopback/replay.cpp) as synchronous calls and inside batch
              scopes with host deferral (ecg_batch_defer_host), beside the CPU baseline's per-stripe calls.

Multi-GPU: one process per GPU (torch.distributed.run), stripes sharded per rank (ecg_dist), no
data-path collective: rank 0's coding plan broadcast before the run, barrier + synchronize around the
timed region, elapsed time max-reduced, per-rank parity checksums all-gathered.  `--gpus N` with N > 1
outside a torch.distributed environment starts N fresh rank processes itself (torch.distributed.run as a
child process, before anything touches the GPU), relays rank 0's JSON line and exits with the ranks'
status; inside one, N must equal WORLD_SIZE.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (importing torch does not initialise the GPU)

import ecg  # noqa: E402  (loads libecg.so lazily, on first use)
import ecg_dist as D  # noqa: E402
from ecg_ring import (azure_local_split, global_ring_state, pc_merge_ring_state,  # noqa: E402
                      ring_repair_state)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
REPLAY_THREADS = (4, 8, 16)  # lrc-repair: concurrent host threads issuing the per-call reference sequence
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")
METRIC = "GiB/s encode + single-block decode (device-resident), RS(10,4) 1 MiB blocks, 1 & 8 GPU"
# BASELINE.json configs[4]: RS(10,4), 4 MiB blocks, 65536 stripes sharded over the GPUs, encoded in
# HBM-resident waves of 1024 stripes.  Its combined parity checksum does not depend on the sharding; the
# N = 1 value of the full batch (profiles/r02/workloads/bench_rs4m-waves.log) is the bit-exact check at N > 1.
CONFIG5_STRIPES, CONFIG5_BLOCK, CONFIG5_WAVE = 65536, 4 << 20, 1024
CONFIG5_CHECKSUM_N1 = 0x3B120CA5EC06F46F
LAUNCH_TIMEOUT_S = 1200.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks (default: WORLD_SIZE under torch.distributed.run, else 1)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="rs-encode-decode",
                    choices=["rs-encode-decode", "rs-decode-patterns", "lrc-repair", "lrc-repair-ring", "lrc-global-ring",
                             "pc-merge", "pc-merge-ring",
                             "rs4m-waves", "rs-host", "rs-small-host", "families"])
    ap.add_argument("--stripes", type=int, default=None, help="stripes per GPU (default per workload)")
    ap.add_argument("--block-size", type=int, default=None)
    ap.add_argument("--chunk", type=int, default=None, help="lrc-repair-ring: stripes per transfer")
    ap.add_argument("--forms", default=None,
                    help="lrc-repair: comma-separated subset of its forms (default: all), e.g. for a profile")
    ap.add_argument("--self-p2p", action="store_true",
                    help="lrc-repair-ring at N = 1: rank 0 sends the partials to itself over RCCL point to point "
                         "(the N > 1 nccl code path on one GPU; the rate is an intra-GPU copy, not xGMI)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--launch-check", action="store_true",
                    help="rank bookkeeping only (gloo, no GPU): each rank reports itself, rank 0 prints one line")
    ap.add_argument("--no-config5", action="store_true",
                    help="default workload: skip the config-5 sub-object (RS(10,4) 4 MiB waves) of the line")
    ap.add_argument("--config5-stripes", type=int, default=CONFIG5_STRIPES,
                    help="config 5's global stripe count, sharded over the ranks (BASELINE: 65536)")
    ap.add_argument("--config5-block-size", type=int, default=CONFIG5_BLOCK)
    ap.add_argument("--no-host-path", action="store_true",
                    help="default workload: skip the host-path sub-object (pinned host batch incl. PCIe copies)")
    ap.add_argument("--no-families", action="store_true",
                    help="default workload: skip the families sub-object (every code class through the facade)")
    ap.add_argument("--no-configs34", action="store_true",
                    help="default workload: skip the config3 / config4 sub-objects (LRC repair, PC merge on one GPU)")
    ap.add_argument("--configs34-stripes", type=int, default=None,
                    help="default workload: stripes (config 3) / merges (config 4) per GPU (default 4096 / 512)")
    ap.add_argument("--working-set-gib", type=float, default=4.0,
                    help="families: stripes per class so the stripes take at least this many GiB (default 4)")
    ap.add_argument("--ring-scale", type=float, default=1.0,
                    help="default workload: scale the cross-GPU objects' stripe / merge counts (rehearsals of many "
                         "ranks on one GPU)")
    ap.add_argument("--no-ring", action="store_true",
                    help="default workload: skip the cross-GPU partial-decoding object (ring_repair)")
    ap.add_argument("--timeout", type=float, default=LAUNCH_TIMEOUT_S,
                    help="--gpus N > 1 started outside torch.distributed: wall-clock limit (s) on the ranks; "
                         "past it every rank is killed and bench.py exits 124")
    return ap.parse_args()


def launch_ranks(a) -> int:
    """`--gpus N` (N > 1) without a torch.distributed environment: start N fresh rank processes with
    torch.distributed.run as a CHILD process (this process never touches the GPU and never exec()s),
    forward their output, relay rank 0's JSON line on stdout, and return non-zero if any rank failed or
    rank 0 printed no line.  Each rank re-runs this file with the same arguments; it sees WORLD_SIZE = N.

    Watchdog: the child runs in its own process group; if it is still running after `--timeout` seconds
    (a rank stuck in RCCL init or a collective, a hung kernel), the whole group gets SIGTERM, then SIGKILL
    10 s later, and this returns 124.  The ranks' own limit is ecg_dist's init/collective timeout."""
    import signal
    import socket
    import subprocess
    import threading
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, start_new_session=True)
    fired = threading.Event()

    def kill_group(sig):
        try:
            os.killpg(p.pid, sig)  # the group this call started (start_new_session: pgid == p.pid)
        except ProcessLookupError:
            pass

    def expire():
        if p.poll() is None:
            fired.set()
            print(f"bench.py: ranks still running after {a.timeout:.0f} s: terminating them", file=sys.stderr)
            kill_group(signal.SIGTERM)
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                kill_group(signal.SIGKILL)

    timer = threading.Timer(a.timeout, expire)
    timer.daemon = True
    timer.start()
    lines = []
    try:
        for ln in p.stdout:
            if ln.startswith("{"):
                lines.append(ln.strip())
            else:
                sys.stderr.write(ln)
                sys.stderr.flush()
        rc = p.wait()
    finally:
        timer.cancel()
    if fired.is_set():
        return 124
    if rc != 0:
        print(f"bench.py: {a.gpus} ranks under torch.distributed.run exited with status {rc}", file=sys.stderr)
        return rc
    if len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


def events(n):
    return [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(n)]


def timed_loop(r, steps, step):
    """barrier + synchronize, K steps (each records its own events), synchronize + barrier; max over ranks."""
    evs = events(steps)
    D.barrier(r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(evs[i])
    torch.cuda.synchronize()
    D.barrier(r)
    elapsed = time.perf_counter() - t0
    return D.max_over_ranks(elapsed, r, device="cuda"), evs


def warm_for(fn, count, seconds=0.03, chunk=4):
    """At least `count` untimed calls of fn, and more, `chunk` at a time with a synchronize after each, until
    `seconds` of wall time have passed; returns the calls made.  A row that follows host-side setup (a class's
    repair plans, its decode dependency probe, the previous class's oracle check) starts on a nearly idle GPU,
    and two 1 ms batches did not bring its clocks back: the families encodes ran 3-15 % below the same launch
    run back to back."""
    t0 = time.perf_counter()
    i = 0
    while i < count or time.perf_counter() - t0 < seconds:
        for _ in range(chunk):
            fn()
        i += chunk
        torch.cuda.synchronize()
    return i


def pipelined_loop(r, steps, step):
    """barrier + synchronize, ONE untimed pre-roll step, then K steps (each records its own events), synchronize +
    barrier; max over ranks.  The pre-roll keeps the GPU busy while the host records the first timed step, as it is
    in a continuous stream of batches: every timed step's events then span max(GPU time, host time) of its batch,
    not the first batch's host recording on an idle GPU.  step(None) is the pre-roll.  The wall time covers
    K + 1 steps."""
    evs = events(steps)
    D.barrier(r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step(None)
    for i in range(steps):
        step(evs[i])
    torch.cuda.synchronize()
    D.barrier(r)
    elapsed = time.perf_counter() - t0
    return D.max_over_ranks(elapsed, r, device="cuda"), evs


PROFILE_FILE = os.path.join(ROOT, "profiles", "headline_profile.json")


def libecg_sha16():
    import hashlib
    with open(os.path.join(ROOT, "erasure-codes-prototype_amd", "lib", "libecg.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def build_provenance():
    """The libecg.so this run loads, the sources in this tree, and the record __graft_entry__.build() left
    (lib/build_info.json): whether this .so is the one build() produced from exactly these sources."""
    out = {"libecg_sha16": libecg_sha16()}
    try:
        import __graft_entry__ as G
        out["sources_sha16"] = G.sources_sha16()
        info = json.load(open(os.path.join(ROOT, "erasure-codes-prototype_amd", "lib", "build_info.json")))
        out["build_info"] = info
        out["built_by_build_from_these_sources"] = (info.get("libecg_sha16") == out["libecg_sha16"] and
                                                    info.get("sources_sha16") == out["sources_sha16"])
    except Exception as e:  # noqa: BLE001 -- no record: the line says so
        out["build_info"] = None
        out["note"] = f"{type(e).__name__}: {str(e)[:120]}"
    return out


def committed_profile():
    """The committed headline-only rocprofv3 summary (tools/profile_summary.py) and PMC file, named beside
    this run's HIP-event fractions, with whether they were taken on this very libecg.so build."""
    out = {}
    try:
        prof = json.load(open(PROFILE_FILE))
        me = libecg_sha16()
        out = {"profile_kernel_avg_ms": prof["encode"]["avg_ms"], "profile_frac": prof["encode"]["frac_avg"],
               "profile_decode_avg_ms": prof["decode"]["avg_ms"], "profile_decode_frac": prof["decode"]["frac_avg"],
               "profile_source": "profiles/headline_profile.json <- " + prof["source"],
               "profile_libecg_sha16": prof["libecg_sha16"], "profile_is_this_build": prof["libecg_sha16"] == me}
        pm = json.load(open(PMC_FILE))
        out["traffic_libecg_sha16"] = pm.get("libecg_sha16")
        out["traffic_is_this_build"] = pm.get("libecg_sha16") == me
    except Exception:  # noqa: BLE001 -- no committed profile: the line says so
        out.setdefault("profile_source", None)
    return out


def pmc_traffic(tag, workload_key):
    if os.path.exists(PMC_FILE):
        try:
            pm = json.load(open(PMC_FILE))
            if pm.get("workload") == workload_key:
                return pm.get(f"{tag}_hbm_bytes_per_launch")
        except Exception:
            return None
    return None


# ------------------------------------------------------------------------------- CPU baseline

def host_cpus():
    """The host CPUs this process may actually use: its affinity set, capped by the cgroup CPU quota
    (cgroup v2 cpu.max "quota period"; the GPU box's job cgroup grants 16 CPUs of a 256-CPU machine, so
    threads beyond the quota only time-slice).  Returns (threads, facts) with the facts stated in the line."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    threads = affinity if quota is None else max(1, min(affinity, int(quota + 0.999)))
    return threads, {"cpu_model": model, "machine_cpus": os.cpu_count(), "affinity_cpus": affinity,
                     "cgroup_cpu_quota": quota}


def cpu_baseline(k, m, B, target_s):
    """Oracle CPU restatement (Jerasure algorithm, gf-complete-style SPLIT(8,4) PSHUFB region multiply)
    of the same step on a bounded sample: encode + single-erasure decode of S_cpu stripes, one
    jerasure call per stripe (proxy.cpp:342-349), one worker thread per host CPU this process may use
    (host_cpus: affinity capped by the cgroup quota)."""
    import numpy as np
    from oracle import ref
    ref.build()
    threads, facts = host_cpus()
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
    line = {"value": round(gib / t_total, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "threads_used": threads, "cores_available": threads,
            "per_thread_GiBps": round(gib / t_total / threads, 3), **facts,
            "sample": f"{reps} x (encode + 1-erasure decode) of {S} RS({k},{m}) stripes x {B} B, "
                      f"one jerasure call per stripe, {threads} host threads, {t_total:.1f} s"}
    aff = facts["affinity_cpus"]
    if aff > threads:
        # the quota caps CPU time, not threads: one thread per CPU of the affinity mask, shown to gain nothing
        S2 = aff
        data2 = np.ascontiguousarray(np.resize(data, (S2, k, B)))
        stripes2 = np.zeros((S2, n, B), np.uint8)
        stripes2[:, :k] = data2
        coding2 = np.zeros((S2, m, B), np.uint8)
        out2 = np.zeros((S2, B), np.uint8)
        reps2, t2 = 0, 0.0
        while t2 < target_s / 3 and reps2 < 100:
            t0 = time.perf_counter()
            ref.encode_batch_mt(k, m, M, data2, coding2, B, S2, aff)
            t1 = time.perf_counter()
            stripes2[:, k:] = coding2
            t_mid = time.perf_counter()
            ref.decode_batch_mt(k, m, M, stripes2, out2, B, S2, aff)
            t2 += (t1 - t0) + (time.perf_counter() - t_mid)
            reps2 += 1
        check = {"threads": aff, "value": round(reps2 * S2 * 2 * k * B / 2 ** 30 / t2, 3), "unit": "GiB/s",
                 "sample": f"{reps2} x (encode + 1-erasure decode) of {S2} stripes, one thread per CPU of the "
                           f"affinity mask, {t2:.1f} s"}
        if check["value"] > line["value"]:  # report whichever thread count the host actually rewards
            quota_run = {key: line[key] for key in ("value", "sample")} | {"threads": threads, "unit": "GiB/s"}
            line.update(value=check["value"], cores=aff, threads_used=aff, cores_available=aff,
                        per_thread_GiBps=round(check["value"] / aff, 3), sample=check["sample"])
            line["quota_threads_check"] = quota_run
        else:
            line["affinity_threads_check"] = check
    return line


# ------------------------------------------------------------------------------- config 2 (default)

def rs_encode_decode(a, r):
    k, m = 10, 4
    B = a.block_size or (1 << 20)
    S = a.stripes or 4096
    n = k + m
    # rank 0 plans (coding matrix, the 14 single-erasure patterns) and fans the plan out (RCCL broadcast)
    M = D.broadcast_ints(ecg.reed_sol_vandermonde_coding_matrix(k, m) if r.rank == 0 else None, r, device="cuda")
    patterns = [[e] for e in D.broadcast_ints(list(range(n)) if r.rank == 0 else None, r, device="cuda")]
    # one HBM arena: the stripes, then the rebuilt blocks right after them.  Where a separate output
    # allocation's pages land set the decode at 0.74-0.83 of HBM; in the stripes' own allocation it ran at
    # 0.78-0.80 (profiles/r03/placement/)
    arena = torch.empty(S * (n + 1) * B, dtype=torch.uint8, device="cuda")
    stripes = arena[:S * n * B].view(S, n, B)
    rebuilt = arena[S * n * B:].view(S, 1, B)
    first = r.rank * S  # weak scaling: rank r holds global stripes [r*S, (r+1)*S)
    ecg.fill_random(stripes, 0xEC0DE, word_offset=D.data_word_offset(first, n, B))
    pattern_of_stripe = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    data, coding = stripes[:, :k], stripes[:, k:]

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
    # the timed steps follow the warm-up with no idle gap (the clocks drop within tens of ms of idle,
    # DESIGN.md §4); the outputs are checked after them -- every step rewrites the same bytes
    elapsed, evs = timed_loop(r, a.steps, step)
    idx = torch.arange(S, device="cuda")
    # outside the timing: the timed decodes rebuilt the erased blocks, and one more decode with every erased
    # block POISONED rebuilds the same bytes (so the kernel neither reads nor copies the block it rebuilds)
    erased = stripes[idx, idx % n].clone()
    assert torch.equal(rebuilt[:, 0], erased), "decode mismatch"
    stripes[idx, idx % n] = 0xA5
    rebuilt.zero_()
    ecg.decode_batch(k, m, M, 1, patterns, stripes, out=rebuilt, pattern_of_stripe=pattern_of_stripe)
    assert torch.equal(rebuilt[:, 0], erased), "decode mismatch with the erased blocks poisoned"
    stripes[idx, idx % n] = erased
    del erased
    checks = D.gather_checksums(D.checksum64(coding.contiguous()), r, device="cuda")
    enc_ms = [e[0].elapsed_time(e[1]) for e in evs]
    dec_ms = [e[1].elapsed_time(e[2]) for e in evs]
    enc_avg = sum(enc_ms) / len(enc_ms) / 1e3
    dec_avg = sum(dec_ms) / len(dec_ms) / 1e3
    enc_bytes = S * (k + m) * B
    dec_bytes = S * (k + 1) * B
    achieved = enc_bytes / enc_avg / 1e9
    value = r.world * S * 2 * k * B * a.steps / elapsed / 2 ** 30
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": r.world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 bytes generated on device)",
        "config": {"workload": f"RS({k},{m}) encode + rotating 1-erasure decode (e = s mod {n})",
                   "block_size": B, "stripes_per_gpu": S, "global_stripes": S * r.world,
                   "parallelism": f"stripes sharded over {r.world} GPU(s), no data-path collective"},
        "encode_gibps_per_gpu": round(S * k * B / enc_avg / 2 ** 30, 2),
        "decode_gibps_per_gpu": round(S * k * B / dec_avg / 2 ** 30, 2),
        "encode_ms": round(enc_avg * 1e3, 3), "decode_ms": round(dec_avg * 1e3, 3),
        "roofline": {"bound": "hbm", "kernel": "gf_vec_kernel<MT=4,STRIDED> (encode)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic("encode", f"rs{k}{m}_B{B}_S{S}"),
                     "traffic_source": "profiles/pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE "
                                       "passes of this bench command (FETCH x2, KiB -> B, per launch), committed "
                                       "with the round's profiles; not measured inside this run",
                     "algorithmic_bytes_per_launch": enc_bytes,
                     "decode_achieved": round(dec_bytes / dec_avg / 1e9, 1),
                     "decode_frac": round(dec_bytes / dec_avg / 1e9 / HBM_PEAK_GBS, 4),
                     "decode_traffic": pmc_traffic("decode", f"rs{k}{m}_B{B}_S{S}"),
                     "frac_source": "HIP events on this run's stream, averaged over the timed steps",
                     **committed_profile()},
        "parity_checksums": [f"{c:016x}" for c in checks],
        "build": build_provenance(),
    }
    # every rank's own kernel times and HBM fractions (HIP events on its stream), not rank 0's only
    mine = [enc_avg * 1e3, dec_avg * 1e3, achieved / HBM_PEAK_GBS, dec_bytes / dec_avg / 1e9 / HBM_PEAK_GBS]
    per = D.gather_floats(mine, r, device="cuda")
    line["per_rank"] = {"encode_ms": [round(x[0], 3) for x in per], "decode_ms": [round(x[1], 3) for x in per],
                        "encode_frac": [round(x[2], 4) for x in per], "decode_frac": [round(x[3], 4) for x in per],
                        "encode_frac_min": round(min(x[2] for x in per), 4),
                        "encode_frac_max": round(max(x[2] for x in per), 4),
                        "decode_frac_min": round(min(x[3] for x in per), 4),
                        "decode_frac_max": round(max(x[3] for x in per), 4)}
    # the headline's buffers go before config 5 allocates its wave
    del arena, stripes, rebuilt, data, coding, pattern_of_stripe, idx, step, evs
    torch.cuda.empty_cache()
    def optional():
        if not a.no_config5:
            line["config5"] = config5(a, r, M, k, m)
        if not a.no_host_path:
            line["host_path"] = host_path_line(a, r, M, k, m)
        if not a.no_configs34:
            line["config3"] = config3_line(a, r)
            line["config4"] = config4_line(a, r)
        if not a.no_families:
            line["families"] = families_line(a, r)
        if not a.no_ring:
            sc = lambda n: max(8, int(n * a.ring_scale)) // 8 * 8  # noqa: E731
            line["ring_repair"] = ring_repair_line(a, r, S=sc(1024))
            line["global_ring_repair"] = ring_repair_line(a, r, S=sc(256), glob=True)
            line["merge_ring"] = merge_ring_line(a, r, S=sc(64))

    optional_section(line, r, ["config5", "host_path", "config3", "config4", "families", "ring_repair",
                               "global_ring_repair", "merge_ring"], optional)
    if r.world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(k, m, B, a.cpu_seconds)
    return line


# ------------------------------------------------------------------------------- configs 3 and 4 in the line

WORKLOAD_PROFILE = os.path.join(ROOT, "profiles", "workload_profile.json")
CONFIG3_FORMS = ("fused", "reference_sequence_scope_scratch", "reference_sequence_per_call",
                 "reference_sequence_per_call_threads8")
CONFIG4_FORMS = ("rows", "fused", "reference_sequence_scope_scratch", "reference_sequence_per_call")


def workload_profile(key):
    """The committed rocprofv3 kernel-trace summary of one form (tools/workload_profile.py ->
    profiles/workload_profile.json): its dominant kernel, that kernel's average launch, the kernels' busy
    time per batch, and whether it was taken on this libecg.so build."""
    try:
        prof = json.load(open(WORKLOAD_PROFILE))
        f = prof["forms"][key]
        return {"kernel": f["dominant_kernel"], "profile_kernel_avg_us": f["dominant_avg_us"],
                "profile_kernel_launches_per_batch": f["dominant_launches_per_batch"],
                "profile_kernel_busy_ms_per_batch": f["kernel_busy_ms_per_batch"],
                "profile_kernel_busy_frac": f["kernel_busy_frac"],
                "profile_source": "profiles/workload_profile.json <- " + f["source"],
                "profile_is_this_build": prof["libecg_sha16"] == libecg_sha16()}
    except Exception:  # noqa: BLE001 -- no committed profile for this form: the object says so
        return {"kernel": None, "profile_source": None}


def seq_cpu_baseline(nb, nout, B, patterns, pat_of, target_s, nscr, S, fill=None):
    """The oracle's CPU restatement of a per-stripe call sequence (ref.call_seq_batch_mt: every call one
    jerasure_matrix_encode with the SIMD split-table region kernels) on a bounded sample of S stripes,
    repeated for about target_s seconds, one worker thread per host CPU this process may use.  Returns
    (seconds, repetitions, threads, host facts, stripes, out)."""
    import numpy as np
    from oracle import ref
    ref.build()
    threads, facts = host_cpus()
    # one stripe of splitmix bytes, the others derived from it by a per-stripe byte (distinct blocks at the
    # cost of one XOR pass: the sample runs to GiBs, and generating it must not outlast the timing)
    base = ref.splitmix_bytes(0xEC0DE, 0, nb * B).reshape(1, nb, B)
    stripes = np.empty((S, nb, B), np.uint8)
    for i in range(S):
        np.bitwise_xor(base[0], np.uint8((37 * i + 11) & 0xFF), out=stripes[i])
    del base
    if fill is not None:
        fill(stripes)
    out = np.zeros((S, nout, B), np.uint8)
    reps, t_total = 0, 0.0
    while t_total < target_s and reps < 1000:
        t0 = time.perf_counter()
        rc = ref.call_seq_batch_mt(stripes, out, patterns, pat_of, nscr, threads)
        t_total += time.perf_counter() - t0
        reps += 1
        if rc < 0:
            raise RuntimeError("oracle call_seq_batch_mt failed")
    return t_total, reps, min(threads, S), facts, stripes, out  # threads the sample's S stripes kept busy


def config3_line(a, r):
    """BASELINE.json configs[2] in the default line: Azure-LRC(12,2,2), 1 MiB, single-block repair of block
    s mod 16 of each of 4096 stripes per GPU with partial decoding (lrc_repair): the fused form, the
    reference's per-stripe call sequence (help_repair's partial, main_repair's partial, perform_addition;
    handle_repair.cpp:246-252,370-376) in batch scopes with the partials declared scratch, and the same
    sequence one call at a time from 1 and 8 host threads.  Each form: HIP-event time, algorithmic and
    executed bytes, the committed profile's kernel, every repaired block verified.  Rank 0 at N = 1 adds the
    oracle's CPU run of the same per-stripe calls."""
    try:
        torch.cuda.empty_cache()
        res = lrc_repair(a, r, only=CONFIG3_FORMS, steps=min(a.steps, 10), warmup=min(a.warmup, 2),
                         S=a.configs34_stripes or 4096, B=1 << 20)
        out = {"workload": "Azure-LRC(12,2,2) single-block repair (block s mod 16), partial_decoding=true, 1 MiB, "
                           f"{res['stripes_per_gpu']} stripes per GPU (BASELINE configs[2])",
               "algorithmic_bytes_per_repair": "(survivors + 1) * B: 7 MiB local, 13 MiB global",
               "algorithmic_bytes_per_batch": res["algorithmic_bytes_per_batch"],
               "local_repairs": res["local_repairs"], "global_repairs": res["global_repairs"], "forms": {}}
        for name, v in res["results"].items():
            out["forms"][name] = {**v, **workload_profile(f"config3/{name}")}
        oks = D.gather_floats([1.0 if all(v["verified"] for v in res["results"].values()) else 0.0], r, device="cuda")
        out["verified_all_ranks"] = all(x[0] == 1.0 for x in oks)
        del res
        torch.cuda.empty_cache()
        if r.world == 1 and r.rank == 0 and not a.no_cpu_baseline:
            out["cpu_baseline"] = config3_cpu_baseline(a)
        return out
    except Exception as e:  # noqa: BLE001 -- reported, the headline stands
        return {"error": f"{type(e).__name__}: {str(e)[:300]}"}


def config3_cpu_baseline(a):
    """The reference's per-stripe repair calls on the CPU over 1 MiB blocks: a local repair is the helper
    partial, the main partial and perform_addition (three jerasure_matrix_encode calls, 1 x 3, 1 x 3, 1 x 2);
    a global-parity repair re-encodes its row from the 12 data blocks.  Stripe s repairs block s mod 16."""
    import numpy as np
    from oracle import ref
    k, g, l, B = 12, 2, 2, 1 << 20
    n = k + g + l
    cp = ecg.CodingParameters(k=k, l=l, g=g, local_or_column=True)
    ec = ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    M = ec.make_encoding_matrix()
    patterns = []
    for e in range(n):
        if e in (12, 13):
            patterns.append([(n, list(range(k)), M[(e - 12) * k:(e - 11) * k])])
            continue
        surv, sets = azure_local_split(e)
        h = ec.partial_decoding_matrix(sets[0], surv, [e])
        mn = ec.partial_decoding_matrix(sets[1], surv, [e])
        patterns.append([(n + 1, sets[0], h), (n + 2, sets[1], mn), (n, [n + 1, n + 2], [1, 1])])
    threads, _ = host_cpus()
    # whole rounds of the 16 patterns, >= 2 per thread up to 16 threads: at most 64 stripes (1 GiB of host
    # blocks) whatever the core count
    t_ = max(1, min(threads, 16))
    S = 2 * n * max(1, (2 * t_ + n - 1) // n)
    pat_of = np.arange(S, dtype=np.int32) % n

    def encode(st):  # the stripes' parities (the repairs read them)
        for s_ in range(st.shape[0]):
            ref.jerasure_matrix_encode_simd(k, g + l, M, [st[s_, j] for j in range(k)],
                                            [st[s_, j] for j in range(k, n)], B)

    t, reps, threads, facts, stripes, out = seq_cpu_baseline(n, 1, B, patterns, pat_of, a.cpu_seconds / 4, 2, S,
                                                             fill=encode)
    local = sum(1 for s_ in range(S) if s_ % n not in (12, 13))
    alg = (local * 7 + (S - local) * 13) * B
    idx = np.arange(S)
    return {"value": round(reps * alg / t / 1e9, 3), "unit": "GB/s of algorithmic bytes ((survivors + 1) * B per repair)",
            "repairs_per_s": round(reps * S / t, 1), "cores": threads, "kind": "port", "threads_used": threads,
            **facts, "verified": bool(np.array_equal(out[:, 0], stripes[idx, idx % n])),
            "sample": f"{reps} x {S} repairs (block s mod 16), the reference's per-stripe calls (helper partial, "
                      f"main partial, perform_addition; global rows re-encoded), {threads} host threads, {t:.1f} s"}


def config4_line(a, r):
    """BASELINE.json configs[3] in the default line: PC(4,1,4,1), 4 MiB blocks, stripe merging x = 2
    (HORIZONTAL), 512 merges per GPU (pc_merge): the row form (each merged row parity one 8 -> 1 XOR launch
    stripe), the fused 40 -> 5 call the engine splits into rows, and the proxies' own per-row sequence
    (helper partial, main partial, perform_addition; merge.cpp:1310-1402) in batch scopes with the partials
    declared scratch and one call at a time.  Rank 0 at N = 1 adds the oracle's CPU run of the same per-row
    call sequence."""
    try:
        torch.cuda.empty_cache()
        res = pc_merge(a, r, only=CONFIG4_FORMS, steps=min(a.steps, 10), warmup=min(a.warmup, 2),
                       S=max(1, a.configs34_stripes // 8) if a.configs34_stripes else 512, B=4 << 20)
        out = {"workload": f"PC(4,1,4,1) merge x=2 horizontal, 4 MiB blocks, {res['merges_per_gpu']} merges per GPU: "
                           "the 5 row parities of the merged PC(8,1,4,1) (BASELINE configs[3])",
               "algorithmic_bytes_per_merge": "5 rows x 9 B = 180 MiB",
               "algorithmic_bytes_per_batch": res["algorithmic_bytes_per_batch"], "forms": {}}
        for name, v in res["results"].items():
            out["forms"][name] = {**v, **workload_profile(f"config4/{name}")}
        oks = D.gather_floats([1.0 if all(v["verified"] for v in res["results"].values()) else 0.0], r, device="cuda")
        out["verified_all_ranks"] = all(x[0] == 1.0 for x in oks)
        del res
        torch.cuda.empty_cache()
        if r.world == 1 and r.rank == 0 and not a.no_cpu_baseline:
            out["cpu_baseline"] = config4_cpu_baseline(a)
        return out
    except Exception as e:  # noqa: BLE001 -- reported, the headline stands
        return {"error": f"{type(e).__name__}: {str(e)[:300]}"}


def config4_cpu_baseline(a):
    """The same merges on the CPU as the proxies compute them: per merged row, the helper's partial and the
    main proxy's partial (jerasure_matrix_encode(4, 1, ones) over each old stripe's 4 row blocks) and
    perform_addition of the two (handle_merge.cpp:269-270,319,453-454; pc_merge_plan), blocks [2][25] per
    merge (PC(4,1,4,1) rowcol2bid, pc.cpp:326-340)."""
    import numpy as np
    B, nb = 4 << 20, 50
    main_blocks, _, _, help_blocks, _, _ = pc_merge_plan(25)
    calls = []
    for row in range(5):
        calls += [(nb + 5, [int(x) for x in help_blocks[row]], [1] * 4),
                  (nb + 6, [int(x) for x in main_blocks[row]], [1] * 4),
                  (nb + row, [nb + 5, nb + 6], [1, 1])]
    threads, _ = host_cpus()
    # 200 MiB of host stripes per merge: the sample is capped at 16 merges (3.2 GiB) whatever the core count
    # (S = threads reached ~55 GiB on a 256-CPU host without a quota); the threads share them
    S = max(1, min(threads, 16))
    t, reps, threads, facts, blocks, out = seq_cpu_baseline(nb, 5, B, [calls], None, a.cpu_seconds / 4, 2, S)
    ok = True
    for row in range(5):
        src = list(main_blocks[row]) + list(help_blocks[row])
        ok &= bool(np.array_equal(out[:, row], np.bitwise_xor.reduce(blocks[:, src], axis=1)))
    return {"value": round(reps * S * 45 * B / t / 1e9, 3), "unit": "GB/s of algorithmic bytes (9 * B per row)",
            "merges_per_s": round(reps * S / t, 1), "cores": threads, "kind": "port", "threads_used": threads,
            **facts, "verified": ok,
            "sample": f"{reps} x {S} merges (per row: helper partial, main partial, perform_addition -- three "
                      f"jerasure_matrix_encode calls), {threads} host threads, {t:.1f} s"}


def optional_deadline_s() -> float:
    """Seconds the line's optional sub-objects (config 5, host path, cross-GPU objects) may take before the
    headline is printed without them (ECG_BENCH_OPTIONAL_DEADLINE_S).  Below the ranks' collective timeout
    (ECG_DIST_TIMEOUT_S), whose watchdog would otherwise end every rank first -- with no line at all."""
    env = os.environ.get("ECG_BENCH_OPTIONAL_DEADLINE_S")
    return float(env) if env else 0.8 * D.timeout_s()


def optional_section(line, r, keys, body):
    """Run body(), which fills line[key] for `keys`, under ecg_dist.deadline: a sub-object that hangs (an
    RCCL exchange across GPUs that never completes, say) must not cost the line the headline measured
    before it.  On expiry rank 0 prints the line with {"error": ...} for every key not filled yet and
    "optional_deadline_hit": true, and every rank exits 0 (the line is valid; the field says it was cut).
    Exceptions inside the sub-objects are caught by the sub-objects themselves.  The watchdog and the main
    thread settle who finishes the section under one lock: once body() has returned the
    watchdog does nothing, and once the watchdog has fired the main thread never prints."""
    import threading
    limit = optional_deadline_s()
    lock = threading.Lock()
    state = {"finished": False}

    def expire():
        with lock:
            if state["finished"]:
                return  # body() returned first: the main thread prints the full line
            state["expired"] = True
        try:
            partial = dict(line)
            for key in keys:
                if key not in partial:
                    partial[key] = {"error": f"not finished within {limit:.0f} s (optional-section deadline, "
                                             "ECG_BENCH_OPTIONAL_DEADLINE_S); the rest of the line stands"}
            partial["optional_deadline_hit"] = True
            if r.rank == 0:
                print(json.dumps(partial), flush=True)
        finally:
            os._exit(0)

    with D.deadline(limit, expire):
        body()
        with lock:
            state["finished"] = True
            expired = state.get("expired", False)
    if expired:  # the watchdog is printing the line and ending the process: never a second line
        threading.Event().wait()


def config5(a, r, M, k, m):
    """BASELINE.json configs[4] inside the default line, at every N: RS(10,4), 4 MiB blocks, 65536 global
    stripes sharded over the ranks as contiguous ranges (D.stripe_range; the coordinator fanning stripes
    out to proxies, repair.cpp:112-132 / proxy.cpp:312-399), encoded in HBM-resident waves of 1024
    stripes whose input is regenerated on device outside the timing (encode_waves).  Aggregate = all
    ranks' data / the slowest rank's summed encode time; every rank's HBM fraction is all-gathered; the
    per-rank parity checksums combine to a value that must equal the N = 1 one."""
    B, total = a.config5_block_size, a.config5_stripes
    n = k + m
    first, last = D.stripe_range(total, r)
    D.barrier(r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_s, checks = encode_waves(k, m, M, B, first, last, CONFIG5_WAVE)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    frac = (last - first) * n * B / kernel_s / 1e9 / HBM_PEAK_GBS if kernel_s > 0 else 0.0
    per = D.gather_floats([last - first, kernel_s, frac, wall], r, device="cuda")
    sums = D.gather_checksums(checks, r, device="cuda")
    t_max = max(x[1] for x in per)
    combined = D.combine(sums)
    full = total == CONFIG5_STRIPES and B == CONFIG5_BLOCK
    return {"workload": f"RS({k},{m}) {B >> 20} MiB encode, {total} stripes over {r.world} GPU(s), "
                        f"waves of {CONFIG5_WAVE} (BASELINE configs[4])",
            "aggregate_GiBps": round(total * k * B / t_max / 2 ** 30, 1) if t_max > 0 else None,
            "encode_seconds_max": round(t_max, 4),
            "wall_seconds_max_incl_regeneration": round(max(x[3] for x in per), 3),
            "stripes_per_rank": [int(x[0]) for x in per],
            "hbm_frac_per_rank": [round(x[2], 4) for x in per],
            "hbm_frac_min": round(min(x[2] for x in per), 4), "hbm_frac_max": round(max(x[2] for x in per), 4),
            "algorithmic_bytes_per_stripe": n * B,
            "parity_checksum": f"{combined:016x}",
            "parity_checksum_n1": f"{CONFIG5_CHECKSUM_N1:016x}" if full else None,
            "checksum_equals_n1": (combined == CONFIG5_CHECKSUM_N1) if full else None}


# ------------------------------------------------------------------------------- config 2, decode detail

def rs_decode_patterns(a, r):
    """RS(10,4), 1 MiB, 4096 stripes: jerasure_matrix_decode (row_k_ones = failed_num, rs.cpp:36) per
    erasure pattern, SURVEY.md §8(d) C2: data loss e=0 (the row_k_ones XOR path: 10 blocks XORed),
    parity loss e=10 (re-encode one row), the rotating single erasure, and 2 / 3 / 4 erasures."""
    k, m = 10, 4
    n = k + m
    B = a.block_size or (1 << 20)
    S = a.stripes or 4096
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 0xEC0DE, word_offset=D.data_word_offset(r.rank * S, n, B))
    ecg.encode_batch(k, m, M, stripes[:, :k], stripes[:, k:])
    out = torch.empty((S, m, B), dtype=torch.uint8, device="cuda")
    rot = (torch.arange(S, device="cuda", dtype=torch.int32) % n).contiguous()
    cases = [("data e=0 (XOR path)", [[0]], None), ("parity e=10", [[10]], None),
             ("rotating single e = s mod 14", [[e] for e in range(n)], rot),
             ("2 erasures {1, 12}", [[1, 12]], None), ("3 erasures {0, 5, 11}", [[0, 5, 11]], None),
             ("4 erasures {2, 3, 7, 13}", [[2, 3, 7, 13]], None)]
    res = {}
    idx = torch.arange(S, device="cuda")
    for name, pats, pos in cases:
        f = len(pats[0])
        o = out[:, :f]

        def step(ev=None, pats=pats, pos=pos, o=o):
            if ev:
                ev[0].record()
            ecg.decode_batch(k, m, M, f, pats, stripes, out=o, pattern_of_stripe=pos)
            if ev:
                ev[1].record()

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        if pos is None:  # written blocks come back in the library's write order (erased data, then coding)
            order = sorted(x for x in pats[0] if x < k) + sorted(x for x in pats[0] if x >= k)
            for i, e in enumerate(order):
                assert torch.equal(o[:, i], stripes[:, e]), f"{name}: block {e} mismatch"
        else:
            assert torch.equal(o[:, 0], stripes[idx, idx % n]), f"{name}: mismatch"
        elapsed, evs = timed_loop(r, a.steps, step)
        t = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs) / 1e3
        alg = S * (k + f) * B  # reads k survivors, writes f blocks
        res[name] = {"ms": round(t * 1e3, 3), "data_GiBps": round(r.world * S * k * B / t / 2 ** 30, 1),
                     "algorithmic_GBps": round(alg / t / 1e9, 1), "algorithmic_frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4)}
    return {"workload": "RS(10,4) 1 MiB decode by erasure pattern, 4096 stripes", "n_gpus": r.world,
            "results": res, "dtype": "u8", "data": "synthetic (splitmix64 bytes generated on device)"}


# ------------------------------------------------------------------------------- config 3

def lrc_repair(a, r, only=None, steps=None, warmup=None, S=None, B=None):
    """Azure-LRC(12,2,2), 1 MiB: every stripe loses block e = s mod 16 and repairs it.
    Data / local-parity loss: local group of 6 survivors.  partial_decoding=true mirrors
    help_repair/main_repair (handle_repair.cpp:249,375,566): helper partial over the survivors in the
    helper partition, main partial over the rest, perform_addition of the two.  The fused form computes
    the repaired block in one launch from the same survivors.  Global-parity loss (12, 13): the global
    path, re-encode from the 12 data blocks (jerasure_matrix_decode re-encodes erased coding rows).
    only: the forms to run (default: --forms, else all); steps / warmup: per form (default: --steps / --warmup)."""
    steps = a.steps if steps is None else steps
    warmup = a.warmup if warmup is None else warmup
    k, l, g = 12, 2, 2
    B = B or a.block_size or (1 << 20)
    S = S or a.stripes or 4096
    n = k + g + l
    cp = ecg.CodingParameters(k=k, l=l, g=g, local_or_column=True)
    ec = ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    M = ec.make_encoding_matrix()  # (g + l) x k
    # block n of every stripe is a slot for the helper's partial in the fused-main form (a helper
    # proxy's partial arriving at the main proxy sits next to the main proxy's own blocks)
    slots = torch.empty((S, n + 1, B), dtype=torch.uint8, device="cuda")
    stripes = slots[:, :n]
    ecg.fill_random(slots, 0xEC0DE, word_offset=D.data_word_offset(r.rank * S, n + 1, B))
    ecg.encode_batch(k, g + l, M, stripes[:, :k], stripes[:, k:])
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    partials = torch.empty((S, 2, B), dtype=torch.uint8, device="cuda")
    e_of = torch.arange(S, device="cuda", dtype=torch.int32) % n
    # helper / main split of every local pattern: azure_local_split
    fused_progs, part_progs, cls_local = [], ([], []), []
    helper_progs, main_progs = [], []  # fused-main form: helper partial -> slot n, main (3 + 1 inputs) -> out
    for e in range(n):
        if e in (12, 13):
            continue
        surv, sets = azure_local_split(e)
        fused_progs.append((ec.partial_decoding_matrix(surv, surv, [e]), surv, [0]))
        for i in range(2):
            part_progs[i].append((ec.partial_decoding_matrix(sets[i], surv, [e]), sets[i], [i]))
        helper_progs.append((ec.partial_decoding_matrix(sets[0], surv, [e]), sets[0], [n]))
        main_row = [list(ec.partial_decoding_matrix(sets[1], surv, [e])) + [1]]
        main_progs.append((main_row, sets[1] + [n], [0]))
        cls_local.append(e)
    # class L launch (6 survivors) over stripes with e not in {12, 13}
    sl = torch.nonzero((e_of != 12) & (e_of != 13)).flatten().to(torch.int32).contiguous()
    lut = torch.full((n,), -1, dtype=torch.int32)
    for i, e in enumerate(cls_local):
        lut[e] = i
    pl = lut.cuda()[e_of[sl].long()].contiguous()
    # class G launch (12 data) over stripes with e in {12, 13}
    sg = torch.nonzero((e_of == 12) | (e_of == 13)).flatten().to(torch.int32).contiguous()
    pg = (e_of[sg.long()] - 12).contiguous()
    glob_progs = [(M[i * k:(i + 1) * k], list(range(k)), [0]) for i in range(g)]

    def step_partial(ev=None):
        if ev:
            ev[0].record()
        for i in range(2):  # the two partials (helper proxies / main proxy)
            ecg.matrix_apply_batch_multi(part_progs[i], stripes, partials, prog_of_stripe=pl, stripe_of=sl)
        ecg.matrix_apply_batch_multi([([[1, 1]], [0, 1], [0])], partials, rebuilt, stripe_of=sl)  # addition
        ecg.matrix_apply_batch_multi(glob_progs, stripes, rebuilt, prog_of_stripe=pg, stripe_of=sg)
        if ev:
            ev[1].record()

    def step_fused_main(ev=None):
        if ev:
            ev[0].record()
        ecg.matrix_apply_batch_multi(helper_progs, slots, slots, prog_of_stripe=pl, stripe_of=sl)  # helper
        ecg.matrix_apply_batch_multi(main_progs, slots, rebuilt, prog_of_stripe=pl, stripe_of=sl)  # main
        ecg.matrix_apply_batch_multi(glob_progs, stripes, rebuilt, prog_of_stripe=pg, stripe_of=sg)
        if ev:
            ev[1].record()

    def step_fused(ev=None):
        if ev:
            ev[0].record()
        ecg.matrix_apply_batch_multi(fused_progs, stripes, rebuilt, prog_of_stripe=pl, stripe_of=sl)
        ecg.matrix_apply_batch_multi(glob_progs, stripes, rebuilt, prog_of_stripe=pg, stripe_of=sg)
        if ev:
            ev[1].record()

    # The reference's own per-stripe call sequence (help_repair's partial, main_repair's partial,
    # perform_addition: handle_repair.cpp:249,371-376,566) on the same blocks, issued from C++ through the
    # C ABI (loopback/replay.cpp), as one call per stripe outside any scope, in deferred-batch scopes, and
    # in scopes with the partials declared scratch (the three calls compose into one region product).
    rp = replay_lib()
    sl_h, pl_h = sl.cpu().to(torch.int32).contiguous(), pl.cpu().to(torch.int32).contiguous()
    n_pat = len(cls_local)
    fail_h = torch.tensor(cls_local, dtype=torch.int32)
    surv_h = torch.tensor([azure_local_split(e)[0] for e in cls_local], dtype=torch.int32).contiguous()
    help_h = torch.tensor([azure_local_split(e)[1][0] for e in cls_local], dtype=torch.int32).contiguous()
    main_h = torch.tensor([azure_local_split(e)[1][1] for e in cls_local], dtype=torch.int32).contiguous()
    assert surv_h.shape == (n_pat, 6) and help_h.shape == main_h.shape == (n_pat, 3)
    part_scratch = torch.empty((sl.numel(), 2, B), dtype=torch.uint8, device="cuda")
    scope_stripes = 512  # tools/scope_repair.cpp's scope size (profiles/r02/scope_repair/)
    replay_stats = {}

    def replay(form):
        def fn(ev=None):
            if ev:
                ev[0].record()
            st = torch.cuda.current_stream().cuda_stream
            rc = rp.ecg_replay_partial_repair(
                ec._h, form, scope_stripes, stripes.data_ptr(), stripes.stride(0), stripes.stride(1), B, sl.numel(),
                sl_h.data_ptr(), pl_h.data_ptr(), fail_h.data_ptr(), 6, surv_h.data_ptr(), 3, help_h.data_ptr(), 3,
                main_h.data_ptr(), part_scratch.data_ptr(), rebuilt.data_ptr(), rebuilt.stride(0), st)
            if rc != 0:
                raise ecg.EcgError(rc, "ecg_replay_partial_repair")
            if form > 0:
                replay_stats[form] = ecg.batch_last_stats()
            ecg.matrix_apply_batch_multi(glob_progs, stripes, rebuilt, prog_of_stripe=pg, stripe_of=sg)
            if ev:
                ev[1].record()
        return fn

    def replay_threads(nthreads):
        """The per-call sequence (form 0) from `nthreads` concurrent host threads, each with its own
        ErasureCode handle and stream over a contiguous share of the repairs (the proxy's thread per
        request, proxy.cpp:416-419).  The worker streams start after and finish before the current stream's
        events, so the events time the whole."""
        import ctypes
        ecs = [ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, cp) for _ in range(nthreads)]
        for e in ecs:
            e.init_coding_parameters(cp)
        streams = [torch.cuda.Stream() for _ in range(nthreads)]
        ec_arr = (ctypes.c_void_p * nthreads)(*[e._h for e in ecs])
        st_arr = (ctypes.c_void_p * nthreads)(*[s.cuda_stream for s in streams])

        def fn(ev=None):
            cur = torch.cuda.current_stream()
            if ev:
                ev[0].record()
            for s_ in streams:
                s_.wait_stream(cur)
            rc = rp.ecg_replay_partial_repair_mt(
                ec_arr, st_arr, nthreads, 0, scope_stripes, stripes.data_ptr(), stripes.stride(0), stripes.stride(1), B,
                sl.numel(), sl_h.data_ptr(), pl_h.data_ptr(), fail_h.data_ptr(), 6, surv_h.data_ptr(), 3,
                help_h.data_ptr(), 3, main_h.data_ptr(), part_scratch.data_ptr(), rebuilt.data_ptr(), rebuilt.stride(0))
            if rc != 0:
                raise ecg.EcgError(rc, "ecg_replay_partial_repair_mt")
            for s_ in streams:
                cur.wait_stream(s_)
            ecg.matrix_apply_batch_multi(glob_progs, stripes, rebuilt, prog_of_stripe=pg, stripe_of=sg)
            if ev:
                ev[1].record()
        fn.keep = (ecs, streams, ec_arr, st_arr)
        return fn

    idx = torch.arange(S, device="cuda")
    results = {}
    n_local, n_glob = sl.numel(), sg.numel()
    alg = (n_local * 7 + n_glob * 13) * B  # (survivors + 1) * B per repair
    per_call_bytes = (n_local * (4 + 4 + 3) + n_glob * 13) * B  # the partials round-trip HBM
    # (name, form factory -- built only when the form runs, executed bytes per batch)
    forms = (("partial_decoding", lambda: step_partial, per_call_bytes),
             ("partial_decoding_fused_main", lambda: step_fused_main, (n_local * (4 + 5) + n_glob * 13) * B),
             ("fused", lambda: step_fused, alg),
             ("reference_sequence_per_call", lambda: replay(0), per_call_bytes),
             ("reference_sequence_scope", lambda: replay(1), per_call_bytes),
             ("reference_sequence_scope_scratch", lambda: replay(2), None),
             *((f"reference_sequence_per_call_threads{t}", (lambda t=t: replay_threads(t)), per_call_bytes)
               for t in REPLAY_THREADS))
    wanted = only if only is not None else (a.forms.split(",") if a.forms else None)
    if wanted is not None:
        forms = tuple(f for f in forms if f[0] in wanted)
    for name, make, executed in forms:
        fn = make()
        rebuilt.zero_()
        warmed = warm_for(fn, warmup)
        assert torch.equal(rebuilt[:, 0], stripes[idx, e_of.long()]), f"{name}: repair mismatch"
        elapsed, evs = pipelined_loop(r, steps, fn)
        t = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs) / 1e3
        res = {"repairs_per_s": round(r.world * S * (steps + 1) / elapsed, 1), "ms_per_batch": round(t * 1e3, 3),
               "algorithmic_GBps": round(alg / t / 1e9, 1), "algorithmic_frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
               "verified": True,  # every repaired block equal to the lost one (the assert above)
               "batches_run": warmed + steps + 1}
        if name == "reference_sequence_scope_scratch":
            st = replay_stats[2]  # the last scope's flush: 3 recorded calls per repair, composed to 1
            res["last_scope_flush"] = st
            per_scope = n_local - ((n_local - 1) // scope_stripes) * scope_stripes  # the last scope's repairs
            composed_away = st["recorded"] == 3 * per_scope and st["composed"] == per_scope and st["materialised"] == 0
            executed = alg if composed_away else None
            res["partials_composed_away"] = composed_away
        elif name == "reference_sequence_scope":
            res["last_scope_flush"] = replay_stats[1]
        if name.startswith("reference_sequence"):
            res["issued_from"] = "C++ through the C ABI (loopback/replay.cpp), one ErasureCode call per step per stripe"
        if "_threads" in name:
            res["issued_from"] += (f"; {name.rsplit('threads', 1)[1]} host threads, each with its own handle and "
                                   "stream over a contiguous share of the repairs")
        res["executed_bytes_per_batch"] = executed
        res["executed_GBps"] = round(executed / t / 1e9, 1) if executed else None
        res["executed_frac"] = round(executed / t / 1e9 / HBM_PEAK_GBS, 4) if executed else None
        results[name] = res
        del fn
    return {"workload": "Azure-LRC(12,2,2) single-block repair, block s mod 16, 1 MiB", "n_gpus": r.world,
            "stripes_per_gpu": S, "steps": steps, "local_repairs": n_local, "global_repairs": n_glob,
            "algorithmic_bytes_per_batch": alg, "results": results, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)"}


_REPLAY = None


def replay_lib():
    """libecg_replay.so (loopback/replay.cpp, built with libecg): the proxies' per-stripe repair and merge
    calls issued from C++ through the C ABI."""
    global _REPLAY
    if _REPLAY is None:
        import ctypes
        path = os.path.join(ROOT, "erasure-codes-prototype_amd", "lib", "libecg_replay.so")
        ecg.lib()  # libecg first (the replay library links it)
        L = ctypes.CDLL(path)
        I, LL, P = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p
        L.ecg_replay_partial_repair.argtypes = [P, I, I, P, LL, LL, I, I, P, P, P, I, P, I, P, I, P, P, P, LL, P]
        L.ecg_replay_partial_repair.restype = I
        L.ecg_replay_partial_repair_mt.argtypes = [P, P, I, I, I, P, LL, LL, I, I, P, P, P, I, P, I, P, I, P, P, P, LL]
        L.ecg_replay_partial_repair_mt.restype = I
        L.ecg_replay_merge.argtypes = [P, P, I, I, P, LL, LL, I, I, I, I, P, P, P, I, P, P, P, P, P, LL, LL, P]
        L.ecg_replay_merge.restype = I
        L.ecg_replay_calls.argtypes = [P, I, I, I, P, LL, LL, I, I, P, P, P, I, I, P, P]
        L.ecg_replay_calls.restype = I
        L.ecg_replay_host_encode.argtypes = [I, I, P, P, P, I, I, I, I]
        L.ecg_replay_host_encode.restype = I
        _REPLAY = L
    return _REPLAY


def merge_ring_line(a, r, S=64, steps=5):
    """The default line's `merge_ring` object: config 4's stripe merging with the old stripes' clusters on
    neighbouring GPUs (pc_merge_ring_state), five 4 MiB row partials per merge over RCCL point to point; at
    N = 1 the rank is its own RCCL peer.  Every new parity is checked; an exception is reported in the
    object instead of failing the headline."""
    B = 4 << 20
    self_p2p = r.world == 1
    try:
        torch.cuda.empty_cache()
        if self_p2p:
            D.init_self_p2p(torch.device("cuda", torch.cuda.current_device()))
        step, out, expected = pc_merge_ring_state(r, S, B, 8, self_p2p=self_p2p)
        out.zero_()
        step()
        torch.cuda.synchronize()
        ok = all(bool(torch.equal(out[i:i + 16], expected(i, min(S, i + 16)))) for i in range(0, S, 16))
        elapsed, _ = timed_loop(r, steps, step)
        oks = D.gather_floats([1.0 if ok else 0.0], r, device="cuda")
        res = {"workload": "PC(4,1,4,1) merge x=2 horizontal, 4 MiB, old stripe 1's cluster on the previous rank: "
                           "five row partials per merge over RCCL point to point, added in the main rank's row launches",
               "backend": D._BACKEND, "self_p2p": self_p2p, "merges_per_gpu": S, "chunk_merges": 8, "steps": steps,
               "merges_per_s": round(r.world * S * steps / elapsed, 1),
               ("rccl_self_GBps" if self_p2p else "xgmi_GBps_per_rank"): round(5 * S * B * steps / elapsed / 1e9, 1),
               "verified_all_ranks": all(x[0] == 1.0 for x in oks)}
        del step, out, expected
        torch.cuda.empty_cache()
        return res
    except Exception as e:  # noqa: BLE001 -- reported, the headline stands
        return {"error": f"{type(e).__name__}: {str(e)[:300]}"}
    finally:
        if self_p2p:
            D.destroy()


def ring_repair_line(a, r, S=1024, steps=5, glob=False):
    """The default line's `ring_repair` object: config 3's partial decoding with the helper and main
    proxies on neighbouring GPUs (lrc_repair_ring below), so that every multi-GPU run of the driver also
    moves partials over RCCL point to point (xGMI) and checks every repaired block.  At N = 1 the one rank
    is its own RCCL peer (ecg_dist.init_self_p2p): the same RCCL code path, the partials copied on the one
    GPU, so each N = 1 run exercises it on hardware too (its GB/s is an on-GPU copy, not xGMI).  An
    exception here is reported in the object instead of failing the headline.  glob: the `global_ring_repair`
    object instead -- global-parity repairs whose four helper partitions sit on ranks q+1 .. q+4
    (global_ring_state): four shifted exchanges per chunk, so at N >= 5 every rank sends on four xGMI links
    and receives on four at once."""
    B = 1 << 20
    self_p2p = r.world == 1
    chunk = 32 if glob else 128
    try:
        torch.cuda.empty_cache()
        if self_p2p:
            D.init_self_p2p(torch.device("cuda", torch.cuda.current_device()))
        state = global_ring_state if glob else ring_repair_state
        step, rebuilt, e_main, main_view = state(r, S, B, chunk, self_p2p=self_p2p)
        rebuilt.zero_()
        step()
        torch.cuda.synchronize()
        lost = main_view[torch.arange(S, device="cuda"), e_main]
        ok = bool(torch.equal(rebuilt[:, 0], lost))
        del lost
        elapsed, _ = timed_loop(r, steps, step)
        oks = D.gather_floats([1.0 if ok else 0.0], r, device="cuda")
        # partials that cross RCCL per repair (global: shifts that land on this rank itself are local copies)
        moved = (sum(1 for d in range(1, 5) if d % r.world) if r.world > 1 else 4) if glob else 1
        out = {"workload": ("Azure-LRC(12,2,2) global-parity repair, 1 MiB, the four helper partitions' partials "
                            "sent from ranks q+1..q+4 over RCCL point to point, added in one launch") if glob else
                           ("Azure-LRC(12,2,2) local repair, 1 MiB, helper partials sent to the next rank over RCCL "
                            "point to point, added in the main rank's fused kernel"),
               "backend": D._BACKEND,  # "nccl" = RCCL over xGMI; "gloo" only in the shared-GPU rehearsal
               "self_p2p": self_p2p,  # N = 1: rank 0 is its own RCCL peer (on-GPU copy, not xGMI)
               "stripes_per_gpu": S, "chunk_stripes": chunk, "steps": steps,
               "repairs_per_s": round(r.world * S * steps / elapsed, 1),
               "partials_over_rccl_per_repair": moved,
               ("rccl_self_GBps" if self_p2p else "xgmi_GBps_per_rank"):
                   round(moved * S * B * steps / elapsed / 1e9, 1),
               "verified_all_ranks": all(x[0] == 1.0 for x in oks)}
        del step, rebuilt, e_main, main_view
        torch.cuda.empty_cache()
        return out
    except Exception as e:  # noqa: BLE001 -- reported, the headline stands
        return {"error": f"{type(e).__name__}: {str(e)[:300]}"}
    finally:
        if self_p2p:
            D.destroy()


def lrc_global_ring(a, r):
    """Config 3's global-parity repairs with the helper proxies on four other GPUs (global_ring_state):
    each repair gathers four 1 MiB partials over RCCL point to point (one exchange of four shifted pairs
    per chunk) and adds them in one launch.  At N = 1 the helpers are local (a copy), or with --self-p2p
    rank 0 is its own RCCL peer for all four."""
    B = a.block_size or (1 << 20)
    S = a.stripes or 256
    moves = r.world > 1 or a.self_p2p
    chunk = max(1, min(S, a.chunk or (32 if moves else S)))
    if a.self_p2p:
        if r.world != 1:
            raise SystemExit("bench.py: --self-p2p is a one-rank mode")
        D.init_self_p2p(torch.device("cuda", torch.cuda.current_device()))
    step, rebuilt, e_main, main_view = global_ring_state(r, S, B, chunk, self_p2p=a.self_p2p)
    rebuilt.zero_()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    lost = main_view[torch.arange(S, device="cuda"), e_main]
    ok = bool(torch.equal(rebuilt[:, 0], lost))
    del lost
    assert ok, "global ring repair mismatch"
    elapsed, evs = timed_loop(r, a.steps, step)
    remote = sum(1 for d in range(1, 5) if d % r.world != 0) if r.world > 1 else (4 if a.self_p2p else 0)
    return {"workload": "Azure-LRC(12,2,2) global-parity repair, 4 helper partitions on the next 4 GPUs, 1 MiB",
            "n_gpus": r.world, "stripes_per_gpu": S, "chunk_stripes": chunk, "steps": a.steps,
            "repairs_per_s": round(r.world * S * a.steps / elapsed, 1),
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "backend": D._BACKEND if moves else None, "self_p2p": bool(a.self_p2p),
            "partials_over_rccl_per_repair": remote,
            "rccl_GBps_per_rank": round(remote * S * B * a.steps / elapsed / 1e9, 1),
            "hbm_algorithmic_bytes_per_repair": 13 * B, "verified": ok, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)"}


def pc_merge_ring(a, r):
    """Config 4's stripe merging with the two old stripes' clusters on neighbouring GPUs (pc_merge_ring_state):
    per merge, 5 row partials of 4 MiB travel over RCCL point to point and the main rank adds them in its
    row launches.  At N = 1 the helper is local (a copy), or with --self-p2p rank 0 is its own RCCL peer."""
    B = a.block_size or (4 << 20)
    S = a.stripes or 64
    moves = r.world > 1 or a.self_p2p
    chunk = max(1, min(S, a.chunk or (8 if moves else S)))
    if a.self_p2p:
        if r.world != 1:
            raise SystemExit("bench.py: --self-p2p is a one-rank mode")
        D.init_self_p2p(torch.device("cuda", torch.cuda.current_device()))
    step, out, expected = pc_merge_ring_state(r, S, B, chunk, self_p2p=a.self_p2p)
    out.zero_()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    ok = all(bool(torch.equal(out[i:i + 16], expected(i, min(S, i + 16)))) for i in range(0, S, 16))
    assert ok, "pc merge ring mismatch"
    elapsed, _ = timed_loop(r, a.steps, step)
    return {"workload": "PC(4,1,4,1) merge x=2 horizontal, 4 MiB, old stripes' clusters on neighbouring GPUs",
            "n_gpus": r.world, "merges_per_gpu": S, "chunk_merges": chunk, "steps": a.steps,
            "merges_per_s": round(r.world * S * a.steps / elapsed, 1),
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "backend": D._BACKEND if moves else None, "self_p2p": bool(a.self_p2p),
            "rccl_GBps_per_rank": round(5 * S * B * a.steps / elapsed / 1e9, 1) if moves else 0.0,
            "hbm_algorithmic_bytes_per_merge": 45 * B, "verified": ok, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)"}


def lrc_repair_ring(a, r):
    """Config 3 with the proxies on different GPUs: cross-GPU partial decoding.

    Azure-LRC(12,2,2), local repairs only (block e = the (s mod 14)-th data / local-parity block of
    stripe s).  Rank q holds S stripes as the MAIN proxy and, for the next rank's S stripes, the
    helper partition's blocks as the HELPER proxy (every rank regenerates the owner's bytes; blocks
    stored block-major, [n + 1][S][B], so the partial slot n of a stripe range is one contiguous
    region).  Per chunk of stripes: the helper-partial kernel (3 survivors -> slot n), RCCL send of the
    chunk's partials to the next rank over xGMI (ring_exchange), and the main rank's fused kernel
    (3 own survivors + the received partial -> repaired block), pipelined so transfers run back to
    back (ecg_dist.pipelined_ring_repair).  One rank: the partial stays in place (no exchange)."""
    B = a.block_size or (1 << 20)
    S = a.stripes or 1024
    # one rank: nothing to overlap, one launch per kernel; N > 1: 128 MiB transfers
    moves = r.world > 1 or a.self_p2p  # the partials cross RCCL
    chunk = max(1, min(S, a.chunk or (128 if moves else S)))
    if a.self_p2p:
        if r.world != 1:
            raise SystemExit("bench.py: --self-p2p is a one-rank mode")
        D.init_self_p2p(torch.device("cuda", torch.cuda.current_device()))
    step, rebuilt, e_main, main_view = ring_repair_state(r, S, B, chunk, self_p2p=a.self_p2p)
    rebuilt.zero_()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    lost = main_view[torch.arange(S, device="cuda"), e_main]
    ok = bool(torch.equal(rebuilt[:, 0], lost))
    del lost
    assert ok, "ring repair mismatch"
    elapsed, evs = timed_loop(r, a.steps, step)
    t = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs) / 1e3
    return {"workload": "Azure-LRC(12,2,2) local repair, helper and main proxies on neighbouring GPUs, 1 MiB",
            "n_gpus": r.world, "stripes_per_gpu": S, "chunk_stripes": chunk, "steps": a.steps,
            "repairs_per_s": round(r.world * S * a.steps / elapsed, 1),
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "ms_per_step_rank0_events": round(t * 1e3, 3),
            "backend": D._BACKEND if moves else None, "self_p2p": bool(a.self_p2p),
            "xgmi_bytes_per_rank_step": S * B if r.world > 1 else 0,
            "xgmi_GBps_per_rank": round(S * B * a.steps / elapsed / 1e9, 1) if r.world > 1 else 0.0,
            "rccl_GBps_per_rank": round(S * B * a.steps / elapsed / 1e9, 1) if moves else 0.0,
            "hbm_executed_bytes_per_rank_step": 9 * S * B, "verified": ok, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)"}


# ------------------------------------------------------------------------------- config 4

def pc_merge_plan(nb=25):
    """The per-row calls of config 4's merge as the proxies issue them (merge.cpp:1310-1402): the old stripes'
    blocks are [2][nb] per merge (PC(4,1,4,1) rowcol2bid, pc.cpp:326-340: data (r<4, c<4) = 4r + c, column
    parity (4, c) = 20 + c).  Row r's helper (help_recal over old stripe 2, a PC(8,1,4,1) handle) takes the
    merged-stripe block ids of its 4 blocks -- columns 4..7 of row r: 8r + 4 + c, or 36 + 4 + c in the
    column-parity row -- and the new row parity's id (32 + r, or 44 = G); the main proxy (main_recal over old
    stripe 1, an RS(8,1) row-code handle) takes columns 0..3 and parity column 8.  Returns int32 arrays
    (main_blocks, main_cols, main_parity, help_blocks, help_ids, help_parity), one row per merged row."""
    import numpy as np

    def old_bid(row, col):
        return row * 4 + col if row < 4 else 20 + col

    def new_bid(row, col):  # PC(8,1,4,1): data 8r + c, R(r) = 32 + r, C(c) = 36 + c, G = 44
        if col == 8:
            return 32 + row if row < 4 else 44
        return row * 8 + col if row < 4 else 36 + col
    rows = range(5)
    main_blocks = [[old_bid(r, c) for c in range(4)] for r in rows]
    help_blocks = [[nb + old_bid(r, c) for c in range(4)] for r in rows]
    help_ids = [[new_bid(r, 4 + c) for c in range(4)] for r in rows]
    arr = lambda x: np.ascontiguousarray(np.array(x, dtype=np.int32))  # noqa: E731
    return (arr(main_blocks), arr([[0, 1, 2, 3]] * 5), arr([8] * 5), arr(help_blocks), arr(help_ids),
            arr([new_bid(r, 8) for r in rows]))


def pc_merge(a, r, only=None, steps=None, warmup=None, S=None, B=None):
    """PC(4,1,4,1), 4 MiB blocks, merge x=2 HORIZONTAL: merged PC(8,1,4,1) row r parity = XOR of the
    two old stripes' row-r data blocks (r < 4) / column-parity blocks (r = 4); the RS(8,1) row code is all
    ones (main_recal / help_recal, handle_merge.cpp:159,269,319,453).  One launch reads 40 blocks and
    writes 5 per merge (the algorithmic minimum, 9 * B per row).  The engine's formulations and the proxies'
    own per-row call sequence are timed (below); only / steps / warmup as in lrc_repair."""
    steps = a.steps if steps is None else steps
    warmup = a.warmup if warmup is None else warmup
    B = B or a.block_size or (4 << 20)
    S = S or a.stripes or 512
    old = ecg.ec_factory(ecg.ECTYPE.PC, ecg.CodingParameters(k1=4, m1=1, k2=4, m2=1))
    nb = old.k + old.m  # 25 blocks per PC(4,1,4,1) stripe
    blocks = torch.empty((S, 2 * nb, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(blocks, 0xEC0DE, word_offset=D.data_word_offset(r.rank * S, 2 * nb, B))
    # rowcol2bid (pc.cpp:326-340) of PC(4,1,4,1): data (r<4, c<4) = 4r + c; column parity (r=4, c<4) = 20 + c
    def bid(row, col):
        return row * 4 + col if row < 4 else 20 + col
    src, coef = [], []
    for row in range(5):
        for half in range(2):
            for col in range(4):
                src.append(half * nb + bid(row, col))
    for row in range(5):
        coef.append([1 if j // 8 == row else 0 for j in range(40)])
    out = torch.empty((S, 5, B), dtype=torch.uint8, device="cuda")
    # "fused": one 40 -> 5 BINARY program per merge (every workgroup streams all 40 blocks).
    # "rows": the row parities are independent 8 -> 1 XORs, so each (merge, row) is its own launch stripe:
    #   program r reads its row's 8 blocks, launch stripe i = (merge i // 5, row i % 5).
    fused = [(coef, src, [0, 1, 2, 3, 4])]
    rows = [([[1] * 8], src[8 * row:8 * row + 8], [row]) for row in range(5)]
    prog_of = (torch.arange(5 * S, device="cuda", dtype=torch.int32) % 5).contiguous()
    stripe_of = (torch.arange(5 * S, device="cuda", dtype=torch.int32) // 5).contiguous()
    def unsplit():  # the fused program as one 40-input launch stripe per merge (ECG_OPT_ROW_SPLIT = 0)
        saved = ecg.get_option(ecg.ECG_OPT_ROW_SPLIT)
        ecg.set_option(ecg.ECG_OPT_ROW_SPLIT, 0)
        try:
            ecg.matrix_apply_batch_multi(fused, blocks, out)
        finally:
            ecg.set_option(ecg.ECG_OPT_ROW_SPLIT, saved)

    # The proxies' own per-row calls (helper partial, main partial, perform_addition; pc_merge_plan), issued
    # from C++ through the C ABI (loopback/replay.cpp ecg_replay_merge): one call at a time (form 0), in
    # deferred-batch scopes (1), and in scopes with the partials declared scratch (2: the three calls compose
    # into the row's one 8 -> 1 product).  The partials buffer is allocated only when such a form runs.
    replay_stats = {}
    scope_merges = 64  # 320 rows, 960 recorded calls per scope

    def replay(form):
        import numpy as np
        rp = replay_lib()
        main_ec = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=8, m=1))
        main_ec.init_coding_parameters(ecg.CodingParameters(k=8, m=1))
        new_cp = ecg.CodingParameters(k1=8, m1=1, k2=4, m2=1)
        help_ec = ecg.ec_factory(ecg.ECTYPE.PC, new_cp)
        help_ec.init_coding_parameters(new_cp)
        plan = pc_merge_plan(nb)
        partials = torch.empty((S, 5, 2, B), dtype=torch.uint8, device="cuda")

        def fn():
            p = [x.ctypes.data for x in plan]
            rc = rp.ecg_replay_merge(main_ec._h, help_ec._h, form, scope_merges, blocks.data_ptr(), blocks.stride(0),
                                     blocks.stride(1), B, S, 5, 4, p[0], p[1], p[2], 4, p[3], p[4], p[5],
                                     partials.data_ptr(), out.data_ptr(), out.stride(0), out.stride(1),
                                     torch.cuda.current_stream().cuda_stream)
            if rc != 0:
                raise ecg.EcgError(rc, "ecg_replay_merge")
            if form > 0:
                replay_stats[form] = ecg.batch_last_stats()
        fn.keep = (main_ec, help_ec, plan, partials, np)
        return fn

    # "fused" is what a multi-row caller reaches: the engine splits the separable 40 -> 5 program into five
    # 8 -> 1 row programs by itself (ECG_OPT_ROW_SPLIT); "fused_unsplit" is the same call without the split
    # (name -> form factory, built only when the form runs)
    variants = {
        "rows": lambda: lambda: ecg.matrix_apply_batch_multi(rows, blocks, out, prog_of_stripe=prog_of,
                                                             stripe_of=stripe_of),
        "fused": lambda: lambda: ecg.matrix_apply_batch_multi(fused, blocks, out),
        "fused_unsplit": lambda: unsplit,
        "reference_sequence_per_call": lambda: replay(0),
        "reference_sequence_scope": lambda: replay(1),
        "reference_sequence_scope_scratch": lambda: replay(2),
    }
    alg = S * 45 * B
    per_call_bytes = S * 5 * 13 * B  # 4 + 1, 4 + 1, 2 + 1 blocks per row: the partials round-trip HBM
    res = {}
    wanted = only if only is not None else (a.forms.split(",") if a.forms else None)
    for name, make in variants.items():
        if wanted is not None and name not in wanted:
            continue
        fn = make()
        def step(ev=None, fn=fn):
            if ev:
                ev[0].record()
            fn()
            if ev:
                ev[1].record()

        out.zero_()
        warmed = warm_for(step, warmup)
        for s in (0, S // 2 + 1, S - 1):  # merges checked against XOR on the host
            hb = blocks[s].cpu().numpy()
            for row in range(5):
                x = 0
                for half in range(2):
                    for col in range(4):
                        x = hb[half * nb + bid(row, col)] ^ x
                assert (out[s, row].cpu().numpy() == x).all(), f"merge mismatch ({name})"
        # every merge of the batch against the XOR of its blocks, on the GPU (the host check above is
        # independent of torch's XOR; this one covers all S merges)
        ok = True
        for s0 in range(0, S, 32):
            s1 = min(S, s0 + 32)
            for row in range(5):
                x = blocks[s0:s1, src[8 * row]].clone()
                for j in src[8 * row + 1:8 * row + 8]:
                    x ^= blocks[s0:s1, j]
                ok &= bool(torch.equal(out[s0:s1, row], x))
            del x
        assert ok, f"merge mismatch ({name}, device check)"
        elapsed, evs = pipelined_loop(r, steps, step)
        t = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs) / 1e3
        executed = alg
        extra = {}
        if name.startswith("reference_sequence"):
            executed = per_call_bytes
            extra["issued_from"] = ("C++ through the C ABI (loopback/replay.cpp ecg_replay_merge), the helper's and "
                                    "the main proxy's partial and perform_addition per merged row")
            if name != "reference_sequence_per_call":
                st = replay_stats[1 if name == "reference_sequence_scope" else 2]
                extra["last_scope_flush"] = st
            if name == "reference_sequence_scope_scratch":
                last = S - ((S - 1) // scope_merges) * scope_merges  # the last scope's merges
                composed_away = (st["recorded"] == 15 * last and st["composed"] == 5 * last
                                 and st["materialised"] == 0)
                extra["partials_composed_away"] = composed_away
                executed = alg if composed_away else None
        res[name] = {"ms_per_batch": round(t * 1e3, 3), "merges_per_s": round(r.world * S * (steps + 1) / elapsed, 1),
                     "algorithmic_GBps": round(alg / t / 1e9, 1),
                     "algorithmic_frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
                     "executed_bytes_per_batch": executed,
                     "executed_frac": round(executed / t / 1e9 / HBM_PEAK_GBS, 4) if executed else None,
                     **extra, "verified": True, "batches_run": warmed + steps + 1}
        del fn
    return {"workload": "PC(4,1,4,1) merge x=2 horizontal, 4 MiB blocks", "n_gpus": r.world,
            "merges_per_gpu": S, "steps": steps, "algorithmic_bytes_per_batch": alg, "results": res,
            "dtype": "u8", "data": "synthetic (splitmix64 bytes generated on device)"}


# ------------------------------------------------------------------------------- every code family

# (name, ECTYPE, coding parameters, the reference's class).  BASELINE's block size, working sets of >= 4 GiB
# per class (far above the 256 MB Infinity Cache).  RS(20,4) / RS(30,4) are the stripes merging x = 2 / 3 RS(10,4)
# stripes produces (merge.cpp:19-449; auxs.cpp:102-120 widens k to x k).
FAMILIES = (
    ("RS(12,4)", 0, dict(k=12, m=4), "rs.cpp:5-76"),
    ("ERS(12,4|x=2,seri_num=1)", 1, dict(k=12, m=4, x=2, seri_num=1), "rs.cpp:282-305"),
    ("Azure_LRC(12,2,2)", 2, dict(k=12, l=2, g=2), "lrc.cpp:576-873"),
    ("Azure_LRC+1(12,3,2)", 3, dict(k=12, l=3, g=2), "lrc.cpp:881-1094"),
    ("Optimal_LRC(12,2,2)", 4, dict(k=12, l=2, g=2), "lrc.cpp:1096-1307"),
    ("Optimal_Cauchy_LRC(12,2,2)", 5, dict(k=12, l=2, g=2), "lrc.cpp:1309-1755"),
    ("Uniform_Cauchy_LRC(12,2,2)", 6, dict(k=12, l=2, g=2), "lrc.cpp:2025-2310"),
    ("PC(4,1,4,1)", 7, dict(k1=4, m1=1, k2=4, m2=1), "pc.cpp:5-551"),
    ("HPC(4,1,4,1|x=2,seri_num=0)", 8, dict(k1=4, m1=1, k2=4, m2=1, x=2, seri_num=0), "pc.cpp:553-867"),
    ("HVPC(4,1,4,1)", 9, dict(k1=4, m1=1, k2=4, m2=1), "pc.cpp:869-1267"),
    ("RS(20,4)", 0, dict(k=20, m=4), "rs.cpp:5-76; merge.cpp:19-449"),
    ("RS(30,4)", 0, dict(k=30, m=4), "rs.cpp:5-76; merge.cpp:19-449"),
)
FAMILY_OPS = ("encode", "repair1", "repair2", "decode2")


def _call(kind, h, ins, outs, a=(), b=(), c=()):
    """One ErasureCode call packed for ecg_replay_calls (loopback/replay.cpp)."""
    return [kind, h, len(ins), *ins, len(outs), *outs, len(a), *a, len(b), *b, len(c), *c]


def _repair_calls(plans, nb):
    """The proxies' partial-decoding repair of one stripe (repair.cpp:192-330 -> handle_repair.cpp): per plan of
    generate_repair_plan, one encode_partial_blocks_for_decoding per cluster's help blocks (handle 1 when the plan
    is local / column, lrc.cpp:32-213, pc.cpp:290-324) into scratch slots, then perform_addition of the partials
    into the failed blocks (written in place).  Returns (calls, scratch slots, algorithmic blocks)."""
    calls, slot, alg = [], nb, 0
    for pl in plans:
        h, fails = (1 if pl.local_or_column else 0), list(pl.failure_idxs)
        f = len(fails)
        surv = [b for grp in pl.help_blocks for b in grp]
        parts = []
        for grp in pl.help_blocks:
            outs = list(range(slot, slot + f))
            slot += f
            calls += _call(1, h, grp, outs, grp, surv, fails)
            parts += outs
        calls += _call(2, h, parts, fails, (len(parts), f))
        alg += len(surv) + f
    return calls, slot - nb, alg


def _pack(progs):
    prog, off = [], [0]
    for p in progs:
        prog += p
        off.append(len(prog))
    return torch.tensor(prog, dtype=torch.int32), torch.tensor(off, dtype=torch.int32)


def _decode_deps(h, k, m, pat):
    """Blocks the degraded-read decode of `pat` depends on (its result is linear in the survivors: survivor i is
    read iff setting every other block to zero and i to random bytes gives nonzero output), on 64-byte host
    blocks.  The algorithmic bytes of the decode are (these + the written blocks) * B."""
    import numpy as np
    n, B = k + m, 64
    deps = []
    rng = np.random.default_rng(len(pat) * 131 + pat[0])
    for i in range(n):
        if i in pat:
            continue
        st = [np.zeros(B, np.uint8) for _ in range(n)]
        st[i][:] = rng.integers(1, 256, B, dtype=np.uint8)
        er = list(pat) + [-1]
        rc = h.decode(st[:k], st[k:], B, er, len(pat))
        if rc != 0:
            raise RuntimeError(f"decode {pat} returned {rc}: {ecg.lib().ecg_last_error()}")
        if any(st[j].any() for j in pat):
            deps.append(i)
    return deps


def families(a, r):
    """Every ErasureCode class of the reference (ec_factory, metadata.cpp:48-77) through the facade, as the proxies
    call it, per stripe, in batch scopes (scratch partials declared, so a repair's partials compose away): four
    operations per class over >= 4 GiB of 1 MiB-block stripes --
      encode   ErasureCode::encode of every stripe (proxy.cpp:346);
      repair1  single-block repair of block s mod n with the class's own generate_repair_plan and partition
               (repair.cpp:22-26): a partial decode per cluster's help blocks + perform_addition;
      repair2  two-block repair (blocks i, i + n/2 of stripe i mod n), same path (run_client.cpp:62-122);
      decode2  degraded-read decode of the same two blocks (ErasureCode::decode, proxy.cpp:666).
    Each row: HIP-event time per batch, algorithmic bytes (encode (k+m) B; repairs (survivors + failed) B per
    plan; decode (blocks the result depends on + written) B) and their fraction of 8 TB/s, the executed bytes
    the library's launches moved (ecg_traffic_counters) over the algorithmic, launches per batch, the launch
    range of the timed batches (tools/families_profile.py maps it to the rocprofv3 kernel trace), and every
    stripe verified: repairs and decodes rebuild poisoned blocks equal to the encoded ones.  --forms filters
    classes by name prefix.  Rank 0 at N = 1 adds a CPU leg per row: the oracle's class restatement of the same
    calls on sampled stripes, timed, and its outputs compared with the GPU's."""
    import ctypes
    B = a.block_size or (1 << 20)
    steps, warmup = a.steps, a.warmup
    want = a.forms.split(",") if a.forms else None
    rp = replay_lib()
    out = {"workload": "families: encode, single- and two-block repair (partial decoding, generate_repair_plan help "
                       "blocks), two-erasure degraded-read decode of every ErasureCode class, 1 MiB blocks",
           "n_gpus": r.world, "block_size": B, "steps": steps, "warmup": warmup, "dtype": "u8",
           "data": "synthetic (splitmix64 bytes generated on device)", "classes": {}}
    for name, t, params, anchor in FAMILIES:
        if want and not any(name.startswith(w) for w in want):
            continue
        torch.cuda.empty_cache()
        try:
            out["classes"][name] = family_rows(a, r, rp, name, t, params, anchor, B, steps, warmup)
        except Exception as e:  # noqa: BLE001 -- reported in the class's row, the other classes still run
            import traceback
            traceback.print_exc()
            out["classes"][name] = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
    fr = [(c, o, v["frac"]) for c, cv in out["classes"].items() for o, v in cv.get("ops", {}).items()]
    out["min_frac"] = min(fr, key=lambda x: x[2]) if fr else None
    out["all_verified"] = all(v["verified"] for cv in out["classes"].values() for v in cv.get("ops", {}).values()) \
        and not any("error" in cv for cv in out["classes"].values())
    out["build"] = build_provenance()
    return out


FAMILIES_PROFILE = os.path.join(ROOT, "profiles", "families_profile.json")


def families_line(a, r):
    """The default line's `families` object: the families workload (every ErasureCode class: encode, single- and
    two-block repair through generate_repair_plan, two-erasure decode; 1 MiB blocks, >= 4 GiB per class, batch
    scopes with scratch partials) at 5 timed batches per row, compacted to one entry per class and operation --
    fraction of 8 TB/s, executed over algorithmic bytes, launches, host time, verified -- with the committed
    rocprofv3 slice of the same row (profiles/families_profile.json: dominant kernel, its average launch, the
    kernels' busy fraction) and the oracle's check of sampled stripes (rank 0 at N = 1)."""
    try:
        torch.cuda.empty_cache()
        fa = argparse.Namespace(**vars(a))
        fa.steps, fa.warmup, fa.forms, fa.stripes, fa.block_size = min(a.steps, 5), min(a.warmup, 2), None, None, None
        res = families(fa, r)
        try:
            prof = json.load(open(FAMILIES_PROFILE))
        except (OSError, ValueError):
            prof = {"classes": {}}
        me = libecg_sha16()
        out = {"workload": res["workload"], "block_size": res["block_size"], "steps": fa.steps,
               "profile_source": "profiles/families_profile.json" if prof["classes"] else None,
               "profile_is_this_build": prof.get("libecg_sha16") == me, "classes": {}}
        for cname, cv in res["classes"].items():
            if "error" in cv:
                out["classes"][cname] = cv
                continue
            rows = {"stripes_per_gpu": cv["stripes_per_gpu"], "working_set_GiB": cv["working_set_GiB"]}
            for op, v in cv["ops"].items():
                pv = prof["classes"].get(cname, {}).get(op, {})
                rows[op] = {"frac": v["frac"], "ms_per_batch": v["ms_per_batch"],
                            "executed_over_algorithmic": v["executed_over_algorithmic"],
                            "launches_per_batch": v["launches_per_batch"], "host_ms_per_batch": v["host_ms_per_batch"],
                            "verified": v["verified"], "kernel": pv.get("dominant_kernel"),
                            "profile_kernel_avg_us": pv.get("dominant_avg_us"),
                            "profile_kernel_busy_frac": pv.get("kernel_busy_frac")}
            if "decode2" in cv:
                rows["decode2"] = cv["decode2"]
            chk = cv.get("cpu_check")
            if chk:
                rows["cpu_check"] = {k: v for k, v in chk.items() if k not in ("sample",)}
            out["classes"][cname] = rows
        out["min_frac"] = res["min_frac"]
        oks = D.gather_floats([1.0 if res["all_verified"] else 0.0], r, device="cuda")
        out["verified_all_ranks"] = all(x[0] == 1.0 for x in oks)
        return out
    except Exception as e:  # noqa: BLE001 -- reported, the headline stands
        return {"error": f"{type(e).__name__}: {str(e)[:300]}"}


def family_rows(a, r, rp, name, t, params, anchor, B, steps, warmup):
    """One class of the families workload: its four operations (see families)."""
    import ctypes
    cp, cpl = ecg.CodingParameters(**params), ecg.CodingParameters(**params, local_or_column=True)
    hG, hL = ecg.ec_factory(t, cp), ecg.ec_factory(t, cpl)
    hG.init_coding_parameters(cp)
    hL.init_coding_parameters(cpl)
    k, m = hG.k, hG.m
    n = k + m
    # the coordinator plans on its own object: generate_repair_plan sets the planning object's local_or_column
    # (lrc.cpp:460-523, pc.cpp:451-551), which would turn hG's later decodes into local ones
    hP = ecg.ec_factory(t, cp)
    hP.init_coding_parameters(cp)
    hP.generate_partition()
    S = a.stripes or -(-int(a.working_set_gib * 2 ** 30) // (n * B))
    S = -(-S // n) * n  # whole rounds of the n single-block patterns
    pats2 = [sorted({i, (i + n // 2) % n}) for i in range(n)]
    pats2 = [p for p in pats2 if hP.check_if_decodable(p)]
    progs = {"encode": ([_call(0, 0, range(k), range(k, n))], [k + m], None)}
    nscr = 0
    for op, pats in (("repair1", [[f] for f in range(n)]), ("repair2", pats2)):
        cl, algs = [], []
        for p in pats:
            ok, plans = hP.generate_repair_plan(p)
            if not ok:
                raise RuntimeError(f"{name}: no repair plan for {p}")
            c, ns, al = _repair_calls(plans, n)
            cl.append(c)
            algs.append(al)
            nscr = max(nscr, ns)
        progs[op] = (cl, algs, pats)
    if t != 1:
        progs["decode2"] = ([_call(3, 0, range(k), range(k, n), list(p) + [-1], [len(p)]) for p in pats2],
                            [len(_decode_deps(hG, k, m, p)) + len(p) for p in pats2], pats2)
    stripes = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(stripes, 0xEC0DE, word_offset=D.data_word_offset(r.rank * S, n, B))
    scratch = torch.empty((S, max(nscr, 1), B), dtype=torch.uint8, device="cuda")
    handles = (ctypes.c_void_p * 2)(hG._h, hL._h)
    truth = None
    cls = {"reference": anchor, "k": k, "m": m, "stripes_per_gpu": S,
           "working_set_GiB": round(S * n * B / 2 ** 30, 2), "ops": {}}
    if t == 1:
        cls["decode2"] = ("not run: EnlargedRSCode inherits RSCode::decode, which decodes with "
                          "reed_sol_vandermonde_coding_matrix(k, m) (rs.cpp:27-42), not the enlarged code's matrix, so the "
                          "reference's degraded read of an ERS stripe does not rebuild it; the facade reproduces those bytes "
                          "(GPU tests against the oracle).  Its repairs use the ERS matrix (rs.cpp:44-66) and run above.")
    for op in FAMILY_OPS:
        if op not in progs:
            continue
        cl, algs, pats = progs[op]
        prog, off = _pack(cl)
        npat = len(cl)
        pat_of = torch.arange(S, dtype=torch.int32) % npat
        alg = sum(algs[s % npat] for s in range(S)) * B
        failed = None
        if pats is not None:
            failed = [(s, b) for s in range(S) for b in pats[s % npat]]
            fs = torch.tensor([x[0] for x in failed], device="cuda")
            fb = torch.tensor([x[1] for x in failed], device="cuda")

        def poison():
            if failed is not None:
                stripes[fs, fb] = 0xA5

        host = [0.0, 0]  # host seconds inside the replay call (recording + flush; launches are asynchronous)

        def fn(ev=None):
            if ev:
                ev[0].record()
            st = torch.cuda.current_stream().cuda_stream
            h0 = time.perf_counter()
            rc = rp.ecg_replay_calls(handles, 2, S, 1, stripes.data_ptr(),  # one scope per batch
                                     stripes.stride(0), stripes.stride(1), B, S, pat_of.data_ptr(), prog.data_ptr(),
                                     off.data_ptr(), n, scratch.shape[1], scratch.data_ptr(), st)
            if rc != 0:
                raise ecg.EcgError(rc, f"ecg_replay_calls({name}, {op})")
            if ev:
                host[0] += time.perf_counter() - h0
                host[1] += 1
                ev[1].record()

        poison()
        warm_for(fn, warmup)
        if op == "encode":
            truth = stripes.clone()
        marks = {}

        def step(ev):
            if ev is not None and "c0" not in marks:
                marks["c0"] = ecg.traffic_counters()  # after the pre-roll's launches: the timed batches' range
            fn(ev)

        elapsed, evs = pipelined_loop(r, steps, step)
        c0, c1 = marks["c0"], ecg.traffic_counters()
        tt = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs) / 1e3
        # the check: a pass that starts from poisoned blocks rebuilds every one of them, nothing else changes
        poison()
        fn()
        torch.cuda.synchronize()
        verified = bool(torch.equal(stripes, truth))
        executed = (c1["bytes"] - c0["bytes"]) / steps
        row = {"ms_per_batch": round(tt * 1e3, 3), "algorithmic_bytes_per_batch": alg,
               "algorithmic_GBps": round(alg / tt / 1e9, 1), "frac": round(alg / tt / 1e9 / HBM_PEAK_GBS, 4),
               "executed_bytes_per_batch": int(executed), "executed_over_algorithmic": round(executed / alg, 4),
               "executed_frac": round(executed / tt / 1e9 / HBM_PEAK_GBS, 4),
               "launches_per_batch": (c1["launches"] - c0["launches"]) / steps,
               "calls_per_batch": sum(_ncalls(cl[s % npat]) for s in range(S)),
               "launch_range": [c0["launches"], c1["launches"]], "verified": verified,
               "host_ms_per_batch": round(host[0] / max(1, host[1]) * 1e3, 3),
               "ops_per_s": round(r.world * S * (steps + 1) / elapsed, 1)}
        if pats is not None:
            row["patterns"] = len(pats)
            row["algorithmic_blocks_per_pattern"] = algs
        cls["ops"][op] = row
    if r.world == 1 and r.rank == 0 and not a.no_cpu_baseline:
        try:
            cls["cpu_check"] = families_cpu_leg(t, params, k, m, B, progs, stripes, truth, n, scratch.shape[1])
        except Exception as e:  # noqa: BLE001 -- reported beside the GPU rows
            cls["cpu_check"] = {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    del stripes, scratch, truth
    return cls


def _ncalls(packed):
    """Calls in one packed call list."""
    i = c = 0
    while i < len(packed):
        n_in = packed[i + 2]
        n_out = packed[i + 3 + n_in]
        q = i + 4 + n_in + n_out
        n_a = packed[q]
        n_b = packed[q + 1 + n_a]
        n_c = packed[q + 2 + n_a + n_b]
        i = q + 3 + n_a + n_b + n_c
        c += 1
    return c


def families_cpu_leg(t, params, k, m, B, progs, stripes, truth, n, nscr):
    """cpu_baseline leg of the families workload: the oracle's restatement of the reference classes
    (oracle/ec_ref.py, region products on its SIMD split-table kernels) runs the same packed calls on sampled
    stripes, one thread, timed; its outputs are the checker of the GPU's stripes (encode: the GPU's parities;
    repairs / decodes: the blocks rebuilt from poisoned ones)."""
    import numpy as np
    from oracle import ec_ref as E
    from oracle import ref as J
    J.build()
    cp, cpl = E.CodingParameters(**params), E.CodingParameters(**params, local_or_column=True)
    oG, oL = E.ec_factory(t, cp), E.ec_factory(t, cpl)
    oG.init_coding_parameters(cp)
    oL.init_coding_parameters(cpl)
    oL.local_or_column = True
    hs = (oG, oL)
    res = {"kind": "port", "cores": 1, "threads_used": 1}
    scalar = J.jerasure_matrix_encode
    J.jerasure_matrix_encode = J.jerasure_matrix_encode_simd  # same semantics, the SIMD region kernels
    try:
        for op in FAMILY_OPS:
            if op not in progs:
                continue
            cl, algs, pats = progs[op]
            npat = len(cl)
            sample = sorted({0, min(k, npat - 1), npat - 1}) if pats is not None else [0]
            t_total, alg, ok = 0.0, 0, True
            for s in sample:
                blocks = [x.copy() for x in truth[s].cpu().numpy()]
                if pats is not None:
                    for b in pats[s % npat]:
                        blocks[b][:] = 0xA5
                else:
                    for b in range(k, n):
                        blocks[b][:] = 0
                scr = [np.zeros(B, np.uint8) for _ in range(nscr)]
                get = lambda i: blocks[i] if i < n else scr[i - n]  # noqa: E731
                packed = cl[s % npat]
                t0 = time.perf_counter()
                i = 0
                while i < len(packed):
                    kind, h, n_in = packed[i], packed[i + 1], packed[i + 2]
                    ins = packed[i + 3:i + 3 + n_in]
                    n_out = packed[i + 3 + n_in]
                    outs = packed[i + 4 + n_in:i + 4 + n_in + n_out]
                    q = i + 4 + n_in + n_out
                    na = packed[q]
                    av = packed[q + 1:q + 1 + na]
                    nb_ = packed[q + 1 + na]
                    bv = packed[q + 2 + na:q + 2 + na + nb_]
                    nc = packed[q + 2 + na + nb_]
                    cv = packed[q + 3 + na + nb_:q + 3 + na + nb_ + nc]
                    i = q + 3 + na + nb_ + nc
                    o = hs[h]
                    I, O = [get(x) for x in ins], [get(x) for x in outs]
                    if kind == 0:
                        o.encode(I, O, B)
                    elif kind == 1:
                        o.encode_partial_blocks_for_decoding(I, O, B, list(av), list(bv), list(cv))
                    elif kind == 2:
                        o.perform_addition(I, O, B, av[0], av[1])
                    elif kind == 3:
                        if o.decode(I, O, B, list(av), bv[0]) != 0:
                            ok = False
                t_total += time.perf_counter() - t0
                alg += algs[s % npat] * B
                ok &= all(np.array_equal(blocks[b], truth[s, b].cpu().numpy()) for b in range(n))
            res[op] = {"GBps": round(alg / t_total / 1e9, 3), "stripes": len(sample), "seconds": round(t_total, 3),
                       "matches_gpu": bool(ok)}
    finally:
        J.jerasure_matrix_encode = scalar
    res["sample"] = ("the same ErasureCode calls on 1-3 stripes per operation through oracle/ec_ref.py (Python "
                     "class restatement over the C oracle's SIMD region multiply), one thread")
    return res


# ------------------------------------------------------------------------------- config 5

def encode_waves(k, m, M, B, first, last, W, seed=0xEC0DE, on_wave=None):
    """Encode global stripes [first, last) of the synthetic RS(k, m) batch in HBM-resident waves of at most
    W stripes ([W][k+m][B] in one buffer).  Each wave's data is regenerated on device from the stripes'
    global splitmix64 offsets (so a stripe's bytes do not depend on the sharding), encoded with ONE
    ecg_encode_batch launch timed by HIP events, and folded into an order-independent parity checksum.
    on_wave(s0, buf) may inspect a wave before the next one overwrites it.  Returns (seconds, checksum)."""
    n = k + m
    wave = torch.empty((min(W, max(1, last - first)), n, B), dtype=torch.uint8, device="cuda")
    ev = events(1)[0]
    kernel_s, checks = 0.0, 0
    for s0 in range(first, last, W):
        buf = wave[:min(W, last - s0)]
        ecg.fill_random(buf, seed, word_offset=D.data_word_offset(s0, n, B))
        ev[0].record()
        ecg.encode_batch(k, m, M, buf[:, :k], buf[:, k:])
        ev[1].record()
        ev[1].synchronize()
        kernel_s += ev[0].elapsed_time(ev[1]) / 1e3
        checks = (checks + D.checksum64(buf[:, k:].contiguous())) & ((1 << 64) - 1)
        if on_wave:
            on_wave(s0, buf)
    del wave
    return kernel_s, checks


def rs4m_waves(a, r):
    """RS(10,4), 4 MiB blocks, 65536 stripes sharded over the ranks; a rank's share (8192 stripes at N=8,
    448 GiB) exceeds HBM, so it is encoded in resident waves of 1024 stripes (56 GiB); each wave's input
    is regenerated on device outside the timed region (tests/test_gpu_parity.py::test_config5_waves runs
    the same code at a small size against the oracle).  The default workload's line carries the same
    measurement as its "config5" object (config5 above)."""
    k, m = 10, 4
    a.config5_stripes = a.stripes or CONFIG5_STRIPES
    a.config5_block_size = a.block_size or CONFIG5_BLOCK
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    return {**config5(a, r, M, k, m), "n_gpus": r.world, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)"}


# ------------------------------------------------------------------------------- host-resident

def rs_small_host(a, r):
    """BASELINE configs[0]'s shape on the GPU: RS(6,4), 1 KiB blocks, one jerasure_matrix_encode per
    stripe on host buffers (the proxy's SET loop, proxy.cpp:312-349), issued from C++ through the C ABI
    (loopback/replay.cpp ecg_replay_host_encode).  Forms: one synchronous call per stripe; the same calls
    in batch scopes with host deferral (ecg_batch_defer_host) of 64 stripes (config 1's object count) and of
    all stripes.  The CPU baseline runs the oracle's per-stripe Jerasure-algorithm encode (SIMD split
    tables) on one host thread over the same bytes (the reference's per-call path); every GPU form's
    parities are compared with its output."""
    import ctypes

    import numpy as np
    k, m = 6, 4
    B = a.block_size or 1024
    S = a.stripes or 4096
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(0xEC0DE + r.rank)
    data = rng.integers(0, 256, (S, k, B), dtype=np.uint8)
    rp = replay_lib()
    mat = (ctypes.c_int * len(M))(*M)

    def gpu(mode, per_scope):
        coding = np.zeros((S, m, B), dtype=np.uint8)
        rc = rp.ecg_replay_host_encode(k, m, mat, data.ctypes.data, coding.ctypes.data, B, S, mode, per_scope)
        if rc:
            raise ecg.EcgError(rc, "ecg_replay_host_encode")
        return coding

    res, outs = {}, {}
    for name, mode, per in (("per_call_sync", 0, 1), ("deferred_scope_64", 1, 64), ("deferred_scope_all", 1, S)):
        gpu(mode, per)  # warm-up (programs, contexts, staging)
        ts = []
        for _ in range(max(1, a.steps)):
            t0 = time.perf_counter()
            outs[name] = gpu(mode, per)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        res[name] = {"us_per_stripe": round(t / S * 1e6, 3), "stripes_per_s": round(S / t, 1),
                     "data_GiBps": round(S * k * B / t / 2 ** 30, 3)}
    same = all(np.array_equal(outs[x], outs["per_call_sync"]) for x in outs)
    line = {"workload": f"RS({k},{m}) {B} B blocks, {S} stripes, one jerasure_matrix_encode per stripe on host "
                        "buffers (BASELINE configs[0] shape), issued from C++", "n_gpus": r.world,
            "results": res, "gpu_forms_identical": same, "dtype": "u8",
            "data": "synthetic (numpy PCG64 bytes, host memory)"}
    if not a.no_cpu_baseline:
        from oracle import ref
        ref.lib()
        cpu_out = np.zeros((S, m, B), dtype=np.uint8)
        ts = []
        for _ in range(max(3, a.steps)):
            t0 = time.perf_counter()
            ref.encode_batch_mt(k, m, M, data, cpu_out, B, S, 1)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        line["cpu_baseline"] = {"us_per_stripe": round(t / S * 1e6, 3), "stripes_per_s": round(S / t, 1),
                                "cores": 1, "kind": "port",
                                "sample": f"{S} stripes, one SIMD split-table jerasure_matrix_encode per stripe, "
                                          "1 thread (the proxy's per-call path)"}
        line["gpu_equals_cpu_baseline"] = bool(np.array_equal(outs["per_call_sync"], cpu_out))
    return line


def rs_host(a, r):
    """RS(10,4), 1 MiB, host-resident (pinned) batch: encode and single-erasure decode including the
    PCIe copies (ecg_encode_batch_host / ecg_decode_batch_host pipelines), chunk size swept."""
    k, m = 10, 4
    n = k + m
    B = a.block_size or (1 << 20)
    S = a.stripes or 512
    M = ecg.reed_sol_vandermonde_coding_matrix(k, m)
    stripes = torch.empty((S, n, B), dtype=torch.uint8).pin_memory()
    dev = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
    ecg.fill_random(dev, 0xEC0DE, word_offset=D.data_word_offset(r.rank * S, n, B))
    stripes.copy_(dev)
    del dev
    torch.cuda.empty_cache()
    out = torch.empty((S, 1, B), dtype=torch.uint8).pin_memory()
    res = {}
    for chunk in (4, 16, 64):
        for name, fn, nbytes in (
                ("encode", lambda: ecg.encode_batch_host(k, m, M, stripes[:, :k], stripes[:, k:], chunk), S * k * B),
                ("decode", lambda: ecg.decode_batch_host(k, m, M, 1, [3], stripes, h_out=out, chunk_stripes=chunk),
                 S * k * B)):
            fn()
            ts = []
            for _ in range(max(2, a.steps // 3)):
                D.barrier(r)
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            t = D.max_over_ranks(min(ts), r, device="cuda")
            res[f"{name}_chunk{chunk}_GiBps"] = round(r.world * nbytes / t / 2 ** 30, 2)
    # the proxy's own buffers are pageable (std::vector / malloc): the same pipeline on ordinary memory
    import numpy as np
    pg = np.empty((S, n, B), np.uint8)
    pg[...] = stripes.numpy()
    pg_out = np.empty((S, 1, B), np.uint8)
    for name, fn in (("encode", lambda: ecg.encode_batch_host(k, m, M, pg[:, :k], pg[:, k:], 16)),
                     ("decode", lambda: ecg.decode_batch_host(k, m, M, 1, [3], pg, h_out=pg_out, chunk_stripes=16))):
        fn()
        ts = []
        for _ in range(max(2, a.steps // 3)):
            D.barrier(r)
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        t = D.max_over_ranks(min(ts), r, device="cuda")
        res[f"pageable_{name}_chunk16_GiBps"] = round(r.world * S * k * B / t / 2 ** 30, 2)
    assert np.array_equal(pg[:, k:], stripes[:, k:].numpy()), "pageable encode mismatch"
    return {"workload": f"RS(10,4) 1 MiB, {S} stripes in pinned host memory, incl. PCIe H2D/D2H",
            "n_gpus": r.world, "results": res, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device, copied to pinned host buffers)"}


def host_path_line(a, r, M, k, m, S=128, chunk=16, runs=3):
    """The default line's `host_path` object: the path as the proxy runs it, starting and ending in host
    memory (north star: the rate including pinned hipMemcpyAsync).  RS(10,4) 1 MiB stripes in pinned host
    memory, encode and single-erasure decode through the H2D -> kernel -> D2H pipelines
    (ecg_encode_batch_host / ecg_decode_batch_host, `chunk` stripes per stage).  Every rank drives its own
    GPU's PCIe link, so at N > 1 the aggregate shows how the links add up.  The encoded parities are
    compared with the device-resident encode of the same bytes.  Reported, never the headline; an
    exception is reported in the object."""
    n, B = k + m, 1 << 20
    try:
        dev = torch.empty((S, n, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(dev, 0xEC0DE, word_offset=D.data_word_offset(r.rank * S, n, B))
        ecg.encode_batch(k, m, M, dev[:, :k], dev[:, k:])
        host = torch.empty((S, n, B), dtype=torch.uint8).pin_memory()
        host[:, :k].copy_(dev[:, :k])
        host[:, k:].zero_()
        out = torch.empty((S, 1, B), dtype=torch.uint8).pin_memory()
        res = {}
        for name, fn in (("encode", lambda: ecg.encode_batch_host(k, m, M, host[:, :k], host[:, k:], chunk)),
                         ("decode", lambda: ecg.decode_batch_host(k, m, M, 1, [3], host, h_out=out,
                                                                  chunk_stripes=chunk))):
            fn()
            ts = []
            for _ in range(runs):
                D.barrier(r)
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            t = D.max_over_ranks(min(ts), r, device="cuda")
            res[f"{name}_GiBps"] = round(r.world * S * k * B / t / 2 ** 30, 2)
        ok = bool(torch.equal(host[:, k:].to("cuda", non_blocking=False), dev[:, k:])) and \
            bool(torch.equal(out[:, 0].to("cuda"), dev[:, 3]))
        oks = D.gather_floats([1.0 if ok else 0.0], r, device="cuda")
        del dev, host, out
        torch.cuda.empty_cache()
        return {"workload": f"RS(10,4) 1 MiB, {S} stripes per GPU in pinned host memory, encode and 1-erasure "
                            f"decode incl. PCIe H2D/D2H ({chunk}-stripe pipeline chunks)",
                **res, "unit": "GiB/s of data (k*B per stripe), all ranks", "verified_all_ranks":
                all(x[0] == 1.0 for x in oks)}
    except Exception as e:  # noqa: BLE001 -- reported, the headline stands
        return {"error": f"{type(e).__name__}: {str(e)[:300]}"}


def launch_check(a, r):
    """--launch-check: the rank bookkeeping of a multi-GPU run without a GPU (gloo): every rank reports its
    rank, local rank and pid; rank 0 prints them (tests/test_dist_cpu.py::test_bench_launcher)."""
    D.init(r, "gloo")
    me = [r.rank, r.local, os.getpid()]
    if r.distributed:
        t = torch.tensor(me, dtype=torch.int64)
        out = [torch.zeros_like(t) for _ in range(r.world)]
        torch.distributed.all_gather(out, t)
        ranks = [x.tolist() for x in out]
    else:
        ranks = [me]
    line = {"metric": METRIC, "n_gpus": r.world, "launch_check": True, "ranks": ranks}
    stall = os.environ.get("ECG_BENCH_TEST_STALL_OPTIONAL")  # fault injection for tests/test_dist_cpu.py only

    def optional():
        if stall is not None and int(stall) == r.rank:
            time.sleep(3600)  # this rank never reaches the collective below
        D.barrier(r)
        line["optional"] = {"ok": True}

    optional_section(line, r, ["optional"], optional)
    return line


def main():
    a = parse()
    if a.gpus is not None and a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    r = D.from_env()
    if a.gpus is not None and a.gpus != r.world:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={r.world}")
    stall = os.environ.get("ECG_BENCH_TEST_STALL_RANK")  # fault injection for tests/test_dist_cpu.py only
    if stall is not None and int(stall) == r.rank:
        time.sleep(3600)  # this rank never joins: the others must fail within ecg_dist's timeout
    if a.launch_check:
        line = launch_check(a, r)
        if r.rank == 0:
            print(json.dumps(line), flush=True)
        if r.distributed:
            torch.distributed.destroy_process_group()
        return
    # ECG_BENCH_SHARED_GPU=1: rehearsal of the N>1 path on a one-GPU box (every rank on cuda:0, gloo
    # for the bookkeeping collectives).  Exercises the rank logic only; its timings mean nothing.
    shared = os.environ.get("ECG_BENCH_SHARED_GPU") == "1"
    dev = 0 if (shared or not r.distributed) else r.local
    torch.cuda.set_device(dev)
    if shared:
        D.init(r, "gloo")
    else:
        D.init(r, "nccl", device=torch.device("cuda", dev) if r.distributed else None)
    ecg.lib().ecg_set_device(torch.cuda.current_device())
    fn = {"rs-encode-decode": rs_encode_decode, "rs-decode-patterns": rs_decode_patterns, "lrc-repair": lrc_repair,
          "lrc-repair-ring": lrc_repair_ring, "lrc-global-ring": lrc_global_ring, "pc-merge": pc_merge,
          "pc-merge-ring": pc_merge_ring,
          "rs4m-waves": rs4m_waves, "rs-host": rs_host, "rs-small-host": rs_small_host, "families": families}[a.workload]
    line = fn(a, r)
    if r.rank == 0:
        print(json.dumps(line), flush=True)
    if r.distributed or D._SELF_P2P:
        D.destroy()


if __name__ == "__main__":
    main()
