#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM bytes for the encode
and decode kernels of bench.py -> profiles/pmc_traffic.json.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half of the bytes
of a wide coalesced 16-B/lane stream, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
Both counters are in KiB.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(pattern):
    per = defaultdict(float)
    names = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per[d] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    return per, names


def main(fetch_glob, write_glob, out, workload):
    f, fn = load(fetch_glob)
    w, wn = load(write_glob)
    import hashlib
    import os
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "erasure-codes-prototype_amd",
                       "lib", "libecg.so")
    res = {"workload": workload, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)",
           "correction": "FETCH_SIZE x2 (gfx950 half-count of 16-B/lane streaming reads); WRITE_SIZE as is; KiB -> B",
           "libecg_sha16": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None}
    for tag, key in (("encode", "gf_vec_kernel<4,"), ("decode", "gf_vec_kernel<1,")):
        fv = [v for d, v in f.items() if key in fn[d].replace(" ", "")]
        wv = [v for d, v in w.items() if key in wn[d].replace(" ", "")]
        if not fv or not wv:
            continue
        fetch = sum(fv) / len(fv) * 1024 * 2
        write = sum(wv) / len(wv) * 1024
        res[f"{tag}_dispatches"] = [len(fv), len(wv)]
        res[f"{tag}_fetch_bytes_per_launch"] = fetch
        res[f"{tag}_write_bytes_per_launch"] = write
        res[f"{tag}_hbm_bytes_per_launch"] = fetch + write
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
