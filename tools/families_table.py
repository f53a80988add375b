#!/usr/bin/env python3
"""Print the families line (and its profile, if given) as a table.  usage: families_table.py LOG [PROFILE_JSON]"""
import json
import sys

line = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
prof = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else {"classes": {}}
for c, cv in line["classes"].items():
    if "error" in cv:
        print(c, cv["error"])
        continue
    for o, v in cv["ops"].items():
        p = prof["classes"].get(c, {}).get(o, {})
        print(f"{c:30s} {o:8s} S={cv['stripes_per_gpu']:4d} ms={v['ms_per_batch']:7.3f} frac={v['frac']:.3f} "
              f"exec/alg={v['executed_over_algorithmic']:.3f} launches={v['launches_per_batch']:5.1f} "
              f"calls={v['calls_per_batch']:5d} host={v.get('host_ms_per_batch')} ok={v['verified']} | {p.get('dominant_kernel')} "
              f"avg={p.get('dominant_avg_us')}us busy={p.get('kernel_busy_frac')}")
