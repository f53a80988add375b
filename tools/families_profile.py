#!/usr/bin/env python3
"""Per-row kernel profile of `bench.py --workload families` -> families_profile.json.

Input: one rocprofv3 --kernel-trace run of the families workload and the JSON line that run printed.  Each row
of the line (class x operation) carries `launch_range` = [l0, l1): the library's region-product launch counter
(ecg_traffic_counters) before and after its timed batches.  The library launches region products only through
launch_gf, in order, from the bench's one thread, so the region kernels of the trace (gf_vec_kernel,
gf_byte_kernel, gf_lat_dword_kernel), ordered by Dispatch_Id, are exactly the counter's launches 0, 1, 2, ...;
the row's kernels are entries l0 .. l1-1.  Per row: the dominant kernel (total time), its average launch, the
kernels' busy time per batch and the fraction of 8 TB/s the row's algorithmic bytes give over it.
usage: families_profile.py TRACE_CSV BENCH_LOG OUT_JSON
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK_GBS = 8000.0
REGION = ("gf_vec_kernel", "gf_byte_kernel", "gf_lat_dword_kernel")


def kernel_name(full):
    n = full[5:] if full.startswith("void ") else full
    n = n.replace("ecg::(anonymous namespace)::", "").replace("ecg::", "")
    return n[:n.index("(")] if "(" in n else n


def main(trace, log, out):
    line = None
    for ln in open(log):
        if ln.startswith("{"):
            line = json.loads(ln)
    rows = []
    for row in csv.DictReader(open(trace)):
        if any(r in row["Kernel_Name"] for r in REGION):
            rows.append((int(row["Dispatch_Id"]), kernel_name(row["Kernel_Name"]),
                         int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    rows.sort()
    steps = line["steps"]
    res = {"what": "rocprofv3 --kernel-trace of bench.py --workload families, kernels sliced per row by the "
                   "library's launch counter", "source": os.path.relpath(trace, ROOT),
           "libecg_sha16": line.get("build", {}).get("libecg_sha16"),
           "region_kernels_in_trace": len(rows), "classes": {}}
    for cname, cv in line["classes"].items():
        res["classes"][cname] = {}
        for op, v in cv["ops"].items():
            l0, l1 = v["launch_range"]
            ks = rows[l0:l1]
            per = {}
            for _, name, d in ks:
                per.setdefault(name, []).append(d)
            busy = sum(d for _, _, d in ks) / steps
            dom = max(per, key=lambda kk: sum(per[kk])) if per else None
            res["classes"][cname][op] = {
                "launches": len(ks), "expected_launches": l1 - l0,
                "dominant_kernel": dom,
                "dominant_avg_us": round(sum(per[dom]) / len(per[dom]) / 1e3, 3) if dom else None,
                "kernels": {kk: {"launches": len(vv), "avg_us": round(sum(vv) / len(vv) / 1e3, 3)}
                            for kk, vv in sorted(per.items(), key=lambda kv: -sum(kv[1]))},
                "kernel_busy_ms_per_batch": round(busy / 1e6, 4),
                "kernel_busy_frac": round(v["algorithmic_bytes_per_batch"] / (busy / 1e9) / 1e9 / HBM_PEAK_GBS, 4)
                if busy else None,
                "bench_event_frac": v["frac"]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
