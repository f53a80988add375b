#!/usr/bin/env python3
"""Per-dispatch SQ counter ratios from a rocprofv3 --pmc counter_collection CSV (one row per counter per
dispatch; values summed over XCDs/SEs).  WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY as fractions of
SQ_WAVE_CYCLES (they partition it, MI355X_MICROARCH.md "rocprofv3 PMC slots"), instructions per wave.

    python tools/sq_summary.py 'gpurun_out/x/pmc_sq/**/*counter_collection.csv' [kernel-substring]
"""
import collections
import csv
import glob
import sys

files = sorted(glob.glob(sys.argv[1], recursive=True))
sub = sys.argv[2] if len(sys.argv) > 2 else "gf_vec"
d = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in files:
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        key = int(r["Dispatch_Id"])
        nm = r["Kernel_Name"]
        names[key] = (nm[nm.find("<"):nm.find(">") + 1] if "<" in nm else nm[:40]) + " grid=" + r["Grid_Size"]
        d[key][r["Counter_Name"]] += float(r["Counter_Value"])
for key in sorted(d):
    s = d[key]
    wc = s.get("SQ_WAVE_CYCLES", 0) or 1
    w = s.get("SQ_WAVES", 0) or 1
    out = [f"{key:4d} {names[key]:32s}"]
    if "SQ_WAVE_CYCLES" in s:
        out.append(f"wave_cyc={wc:.3e}")
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in s:
            out.append(f"{c[3:].lower()}={s[c] / wc:.3f}")
    for c in ("SQ_INSTS_SMEM", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"):
        if c in s:
            out.append(f"{c[9:].lower()}/wave={s[c] / w:.1f}")
    for c in sorted(s):
        if c not in ("SQ_WAVE_CYCLES", "SQ_WAVES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                     "SQ_INSTS_SMEM", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"):
            out.append(f"{c}={s[c]:.3e}")
    print(" ".join(out))
