#!/usr/bin/env python3
"""Per-dispatch summary of a rocprofv3 --kernel-trace CSV: kernels grouped by (name, grid size), so
launches of one kernel with different workgroup counts (e.g. COLS_PER_WG variants) are told apart.

    python tools/trace_summary.py 'gpurun_out/prof/**/*kernel_trace.csv' [name-substring]
"""
import csv
import glob
import statistics
import sys


def main():
    files = sorted(glob.glob(sys.argv[1], recursive=True))
    if not files:
        raise SystemExit(f"no file matches {sys.argv[1]}")
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    groups = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if sub not in name:
                continue
            grid = (row.get("Grid_Size_X") or row.get("Grid_Size", "?"), row.get("Grid_Size_Y", ""))
            dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            groups.setdefault((name, grid), []).append(dur)
    print(f"{'kernel':70s} {'grid':>14s} {'n':>6s} {'avg us':>10s} {'min us':>10s} {'med us':>10s}")
    for (name, grid), d in sorted(groups.items()):
        print(f"{name[:70]:70s} {'x'.join(g for g in grid if g):>14s} {len(d):6d} {statistics.mean(d) / 1e3:10.2f} "
              f"{min(d) / 1e3:10.2f} {statistics.median(d) / 1e3:10.2f}")


if __name__ == "__main__":
    main()
