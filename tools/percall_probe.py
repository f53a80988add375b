#!/usr/bin/env python3
"""Config 4's per-call kernel: the proxies' per-row merge sequence issued one call at a time
(bench.py pc_merge, form reference_sequence_per_call: helper partial 4 -> 1, main partial 4 -> 1,
perform_addition 2 -> 1 per merged row, 4 MiB blocks), under launch-option variants in ONE process.  Each
variant's launch-counter range (ecg_traffic_counters) is printed, so a rocprofv3 --kernel-trace of this run can be
sliced per variant:
    percall_probe.py run                 -> one JSON line (per variant: event fraction, launch range)
    percall_probe.py parse TRACE LOG     -> per variant and kernel: launches, average / median / min duration
Options are speed-only (ecg.h ECG_OPT_*): results never depend on them, and pc_merge checks every merge."""
import json
import os
import statistics
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "erasure-codes-prototype_amd"))

VARIANTS = [  # name, {option: value}; "B=..." variants change the block size (merges scaled to >= 8 GiB)
    ("default", {}),
    ("B=64KiB", {"B": 64 << 10}),
    ("B=1MiB", {"B": 1 << 20}),
    ("B=16MiB", {"B": 16 << 20}),
    ("lds_pad_0", {"ECG_OPT_MT1_LDS_PAD": 0}),
    ("lds_pad_24k", {"ECG_OPT_MT1_LDS_PAD": 24576}),
    ("grid_map_0", {"ECG_OPT_GRID_MAP": 0}),
    ("grid_map_2", {"ECG_OPT_GRID_MAP": 2}),
    ("cols_256", {"ECG_OPT_COLS_PER_WG": 256}),
    ("cols_512", {"ECG_OPT_COLS_PER_WG": 512}),
    ("lat_kernel", {"ECG_OPT_LAT_DWORD_BYTES": 4 << 20}),
    ("nt_loads_only", {"ECG_OPT_NT": 1}),
    ("default_again", {}),
]


def run():
    import torch
    import bench
    import ecg
    import ecg_dist as D
    torch.cuda.set_device(0)
    r = D.from_env()
    ecg.lib().ecg_set_device(0)
    a = types.SimpleNamespace(steps=5, warmup=1, block_size=None, stripes=None, forms=None)
    out = {"what": "pc_merge reference_sequence_per_call, 128 merges x 4 MiB, option variants", "variants": {}}
    for name, opts in VARIANTS:
        opts = dict(opts)
        B = opts.pop("B", 4 << 20)
        S = max(32, (8 << 30) // (50 * B))
        saved = {o: ecg.get_option(getattr(ecg, o)) for o in opts}
        for o, v in opts.items():
            ecg.set_option(getattr(ecg, o), v)
        try:
            c0 = ecg.traffic_counters()
            res = bench.pc_merge(a, r, only=("reference_sequence_per_call",), S=min(S, 4096), B=B)
            c1 = ecg.traffic_counters()
        finally:
            for o, v in saved.items():
                ecg.set_option(getattr(ecg, o), v)
        v = res["results"]["reference_sequence_per_call"]
        out["variants"][name] = {"options": opts, "block_size": B, "algorithmic_frac": v["algorithmic_frac"],
                                 "ms_per_batch": v["ms_per_batch"], "launch_range": [c0["launches"], c1["launches"]],
                                 "bytes_per_launch": (c1["bytes"] - c0["bytes"]) / max(1, c1["launches"] - c0["launches"])}
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def parse(trace, log):
    import csv
    line = [json.loads(x) for x in open(log) if x.startswith("{")][-1]
    rows = []
    for row in csv.DictReader(open(trace)):
        n = row["Kernel_Name"]
        if any(k in n for k in ("gf_vec_kernel", "gf_byte_kernel", "gf_lat_dword_kernel")):
            short = n.replace("void ", "").replace("ecg::(anonymous namespace)::", "")
            rows.append((int(row["Dispatch_Id"]), short[:short.index("(")],
                         int(row["End_Timestamp"]) - int(row["Start_Timestamp"]), int(row["Start_Timestamp"]),
                         int(row["End_Timestamp"])))
    rows.sort()
    res = {}
    for name, v in line["variants"].items():
        l0, l1 = v["launch_range"]
        ks = rows[l0:l1]
        per = {}
        for _, kn, d, _, _ in ks:
            per.setdefault(kn, []).append(d / 1e3)
        gaps = [ks[i + 1][3] - ks[i][4] for i in range(len(ks) - 1)]
        # the sequence per merged row: helper partial 4 -> 1, main partial 4 -> 1, perform_addition 2 -> 1
        pos = {}
        for i, (_, _, d, _, _) in enumerate(ks):
            pos.setdefault(("helper_4to1", "main_4to1", "addition_2to1")[i % 3], []).append(d / 1e3)
        res[name] = {"event_frac": v["algorithmic_frac"], "launches": len(ks), "block_size": v.get("block_size"),
                     "median_gap_us": round(statistics.median(gaps) / 1e3, 3) if gaps else None,
                     "by_call": {p: {"median_us": round(statistics.median(d), 3),
                                     "p10_us": round(sorted(d)[len(d) // 10], 3)} for p, d in pos.items()},
                     "kernels": {kn: {"n": len(d), "avg_us": round(sum(d) / len(d), 3),
                                      "median_us": round(statistics.median(d), 3), "min_us": round(min(d), 3)}
                                 for kn, d in per.items()}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2], sys.argv[3])
