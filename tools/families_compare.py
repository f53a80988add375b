#!/usr/bin/env python3
"""Compare the `frac` of every families row across bench logs.  usage: families_compare.py LOG [LOG ...]"""
import json
import sys

lines = [[json.loads(x) for x in open(p) if x.startswith("{")][-1] for p in sys.argv[1:]]
first = lines[0]
for c, cv in first["classes"].items():
    for op in cv.get("ops", {}):
        vals = []
        for ln in lines:
            v = ln["classes"].get(c, {}).get("ops", {}).get(op)
            vals.append(f"{v['frac']:.3f}" if v else "  -  ")
        print(f"{c:30s} {op:8s} " + "  ".join(vals))
