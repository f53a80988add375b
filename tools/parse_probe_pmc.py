#!/usr/bin/env python3
"""Per-variant PMC counters of tools/placement_probe.py run under `rocprofv3 --kernel-trace --pmc ...`.

The probe's gf_vec_kernel dispatches come in a fixed order: one warm-up launch per variant, then `rounds`
x variants x `reps` timed launches (encode S0, decode S0->R0..R3, encode S1, decode S1->R0..R3).  This maps
each dispatch to its variant by that order and prints, per variant, the kernel-trace duration and every
collected counter (median over the variant's dispatches).
usage: parse_probe_pmc.py <counter_collection.csv> [--rounds 1 --reps 2]
"""
import argparse
import collections
import csv
import statistics

VARIANTS = ["encode S0"] + [f"decode S0->R{i}" for i in range(4)] + ["encode S1"] + [f"decode S1->R{i}" for i in range(4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    per_dispatch = collections.OrderedDict()
    for row in csv.DictReader(open(a.csv)):
        if "gf_vec_kernel" not in row["Kernel_Name"]:
            continue
        d = per_dispatch.setdefault(int(row["Dispatch_Id"]), {"ns": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
        d[row["Counter_Name"]] = float(row["Counter_Value"])
    ids = sorted(per_dispatch)
    # the set-up encodes (one per stripe batch) come first
    order = ["setup"] * 2 + list(VARIANTS) + [v for _ in range(a.rounds) for v in VARIANTS for _ in range(a.reps)]
    if len(ids) != len(order):
        raise SystemExit(f"{len(ids)} gf_vec_kernel dispatches, expected {len(order)}")
    by = collections.defaultdict(list)
    for i, v in zip(ids, order):
        by[v].append(per_dispatch[i])
    names = sorted({k for d in per_dispatch.values() for k in d if k != "ns"})
    print(f"{'variant':16s} {'ms':>7s} " + " ".join(f"{n[:34]:>34s}" for n in names))
    for v in VARIANTS:
        rows = by[v][1:]  # skip the warm-up launch
        ms = statistics.median(r["ns"] for r in rows) / 1e6
        print(f"{v:16s} {ms:7.3f} " + " ".join(f"{statistics.median(r.get(n, 0.0) for r in rows):34.4g}" for n in names))


if __name__ == "__main__":
    main()
