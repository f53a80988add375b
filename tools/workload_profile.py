#!/usr/bin/env python3
"""Config 3 / config 4 form profiles read by bench.py's config3 / config4 objects -> profiles/workload_profile.json.

Each input is one rocprofv3 --kernel-trace run of ONE form (`bench.py --workload lrc-repair --forms F` or
`--workload pc-merge --forms F`, tools/gpu_run.sh step `w34prof`) and the bench line that run printed.  Per
form: every library kernel in the trace (fill_splitmix and one-off launches such as the stripes' initial
encode excluded), the dominant one by total time with its average launch, and the kernels' busy time per
batch, with the fraction of 8 TB/s the form's algorithmic bytes give over that busy time.  The bench
line's HIP-event fraction divides by the batch's wall time instead, so for the per-call forms (a launch
per call, gaps between kernels) the busy fraction is the higher of the two.
usage: workload_profile.py OUT_JSON KEY=TRACE_CSV:BENCH_LOG:FORM [...]     (KEY e.g. config3/fused)
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK_GBS = 8000.0


def sha16(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def kernel_name(full):
    """'void ecg::(anonymous namespace)::gf_vec_kernel<1, 2, 3, true>(ecg::GfLaunch)' -> 'gf_vec_kernel<1, 2, 3, true>'"""
    n = full[5:] if full.startswith("void ") else full
    n = n.replace("ecg::(anonymous namespace)::", "").replace("ecg::", "")
    return n[:n.index("(")] if "(" in n else n


def bench_line(log):
    line = None
    for ln in open(log):
        if ln.startswith("{"):
            line = json.loads(ln)
    return line


def summarise(trace, log, form):
    line = bench_line(log)
    res = line["results"][form]
    batches = res["batches_run"]
    alg = line["algorithmic_bytes_per_batch"]
    per = {}
    for row in csv.DictReader(open(trace)):
        name = row["Kernel_Name"]
        if "ecg::" not in name or "fill_splitmix" in name:
            continue
        short = kernel_name(name)
        per.setdefault(short, []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    per = {k: v for k, v in per.items() if len(v) > 1}  # one-off setup launches
    busy = sum(sum(v) for v in per.values())
    dom = max(per, key=lambda k: sum(per[k]))
    d = per[dom]
    stats = os.path.join(os.path.dirname(trace), "run_kernel_stats.csv")
    return {"source": os.path.relpath(trace, ROOT) + " (summarised on the box; the trace is not kept)",
            "kernel_stats": os.path.relpath(stats, ROOT), "bench_log": os.path.relpath(log, ROOT), "batches": batches,
            "algorithmic_bytes_per_batch": alg,
            "kernels": {k: {"launches": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 3),
                            "min_us": round(min(v) / 1e3, 3), "total_ms": round(sum(v) / 1e6, 3)}
                        for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))},
            "dominant_kernel": dom, "dominant_avg_us": round(sum(d) / len(d) / 1e3, 3),
            "dominant_launches_per_batch": round(len(d) / batches, 2),
            "kernel_busy_ms_per_batch": round(busy / batches / 1e6, 4),
            "kernel_busy_frac": round(alg / (busy / batches / 1e9) / 1e9 / HBM_PEAK_GBS, 4),
            "bench_event_frac": res["algorithmic_frac"]}


def main(out, *specs):
    lib = os.path.join(ROOT, "erasure-codes-prototype_amd", "lib", "libecg.so")
    res = {"what": "rocprofv3 --kernel-trace of bench.py --workload lrc-repair / pc-merge, one run per form",
           "libecg_sha16": os.environ.get("ECG_PROFILED_LIBECG_SHA16") or sha16(lib),  # run on the profiled tree
           "bench_sha16": sha16(os.path.join(ROOT, "bench.py")), "forms": {}}
    for spec in specs:
        key, rest = spec.split("=", 1)
        trace, log, form = rest.split(":")
        res["forms"][key] = summarise(trace, log, form)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
