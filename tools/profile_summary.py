#!/usr/bin/env python3
"""Headline profile summary read by bench.py's roofline object -> profiles/headline_profile.json.

Inputs: the rocprofv3 --kernel-trace CSV of `bench.py --no-config5 --no-ring --no-host-path --no-configs34` (the headline
alone, so the encode / decode instantiations run nothing else) and the PMC traffic JSON of the same tree
(tools/parse_pmc.py).  Output: per-kernel average and median launch durations over every launch in the
trace, the fractions of 8 TB/s they give for the algorithmic bytes, the PMC bytes, and the sha256 prefixes
of the libecg.so and bench.py that were profiled, so a bench line can say whether the committed profile
is of its own build.
usage: profile_summary.py TRACE_CSV PMC_JSON OUT_JSON [STEPS]
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK_GBS = 8000.0
ENC_BYTES = 4096 * 14 * (1 << 20)  # RS(10,4) encode, S = 4096, 1 MiB: (k + m) B per stripe
DEC_BYTES = 4096 * 11 * (1 << 20)  # rotating single-erasure decode: (k + 1) B per stripe
KERNELS = (("encode", "gf_vec_kernel<4, 2, 3, false>", ENC_BYTES), ("decode", "gf_vec_kernel<1, 2, 3, false>", DEC_BYTES))


def sha16(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def main(trace, pmc, out, steps=None):
    rows = list(csv.DictReader(open(trace)))
    res = {"source": os.path.relpath(trace, ROOT), "what": "rocprofv3 --kernel-trace of bench.py --no-config5 --no-ring "
           "--no-host-path (headline kernels only); every launch in the trace (warm-up included)",
           "libecg_sha16": sha16(os.path.join(ROOT, "erasure-codes-prototype_amd", "lib", "libecg.so")),
           "bench_sha16": sha16(os.path.join(ROOT, "bench.py"))}
    if steps:
        res["bench_steps"] = int(steps)
    pm = json.load(open(pmc)) if pmc and os.path.exists(pmc) else {}
    for tag, name, alg in KERNELS:
        d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
                   if r["Kernel_Name"].startswith(f"void ecg::(anonymous namespace)::{name}"))
        if not d:
            continue
        avg = sum(d) / len(d)
        med = d[len(d) // 2]
        res[tag] = {"launches": len(d), "avg_ms": round(avg / 1e6, 4), "median_ms": round(med / 1e6, 4),
                    "min_ms": round(d[0] / 1e6, 4), "algorithmic_bytes_per_launch": alg,
                    "frac_avg": round(alg / (avg / 1e9) / 1e9 / HBM_PEAK_GBS, 4),
                    "frac_median": round(alg / (med / 1e9) / 1e9 / HBM_PEAK_GBS, 4),
                    "pmc_hbm_bytes_per_launch": pm.get(f"{tag}_hbm_bytes_per_launch")}
    res["pmc_source"] = os.path.relpath(pmc, ROOT) if pmc else None
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
