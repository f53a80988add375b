#!/usr/bin/env python3
"""HBM traffic per row of `bench.py --workload families` from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
-> families_pmc.json.  Corrections as tools/parse_pmc.py (MI355X_MICROARCH.md, HBM section): FETCH_SIZE x2 for
16-B/lane streaming reads, WRITE_SIZE as is, KiB -> B.  Rows are sliced as tools/families_profile.py does: the
library's region kernels in dispatch order are its launch counter's launches, each row names its [l0, l1).
Each pass is its own run of the same command, so each pass's log gives its own launch ranges.
usage: families_pmc.py FETCH_GLOB FETCH_LOG WRITE_GLOB WRITE_LOG OUT_JSON"""
import csv
import glob
import json
import sys
from collections import defaultdict

REGION = ("gf_vec_kernel", "gf_byte_kernel", "gf_lat_dword_kernel")


def per_dispatch(pattern):
    val, name = defaultdict(float), {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in REGION):
                d = int(r["Dispatch_Id"])
                val[d] += float(r["Counter_Value"])
                name[d] = r["Kernel_Name"]
    ids = sorted(val)
    return [val[d] for d in ids], [name[d] for d in ids]


def line(log):
    return [json.loads(x) for x in open(log) if x.startswith("{")][-1]


def main(fetch_glob, fetch_log, write_glob, write_log, out):
    fv, _ = per_dispatch(fetch_glob)
    wv, _ = per_dispatch(write_glob)
    lf, lw = line(fetch_log), line(write_log)
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate runs of bench.py --workload families",
           "correction": "FETCH_SIZE x2; WRITE_SIZE as is; KiB -> B",
           "libecg_sha16": lf.get("build", {}).get("libecg_sha16"), "steps": lf["steps"], "classes": {}}
    for cname, cv in lf["classes"].items():
        if "ops" not in cv:
            continue
        res["classes"][cname] = {}
        for op, v in cv["ops"].items():
            a0, a1 = v["launch_range"]
            b0, b1 = lw["classes"][cname]["ops"][op]["launch_range"]
            fetch = sum(fv[a0:a1]) * 1024 * 2 / lf["steps"]
            write = sum(wv[b0:b1]) * 1024 / lw["steps"]
            alg = v["algorithmic_bytes_per_batch"]
            res["classes"][cname][op] = {"fetch_bytes_per_batch": fetch, "write_bytes_per_batch": write,
                                         "hbm_bytes_per_batch": fetch + write, "algorithmic_bytes_per_batch": alg,
                                         "hbm_over_algorithmic": round((fetch + write) / alg, 4),
                                         "kernels": [a1 - a0, b1 - b0]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
