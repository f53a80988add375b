#!/usr/bin/env python3
"""Print the families line (and its profile, if given) as a table.
  usage: families_table.py LOG [PROFILE_JSON]
         families_table.py --markdown LOG_BOX0 LOG_BOX1 PROFILE_JSON PMC_JSON [CAUSES_JSON]
The markdown form is DESIGN.md §4f's table: one row per class x operation with the fraction of 8 TB/s on both
boxes' default lines, the kernels' busy fraction and the dominant kernel from the rocprofv3 slice of the row, the
PMC HBM bytes over algorithmic, launches and host / GPU time per batch, and the cause codes (CAUSES_JSON:
{"class/op": "codes"}) of every row below 0.70 on either box."""
import json
import sys


def line_of(path):
    rows = [json.loads(x) for x in open(path) if x.startswith("{")]
    line = rows[-1]
    return line["families"] if "families" in line else line


def markdown(a_path, b_path, prof_path, pmc_path, causes_path=None):
    a, b = line_of(a_path)["classes"], line_of(b_path)["classes"]
    prof = json.load(open(prof_path))["classes"]
    pmc = json.load(open(pmc_path))["classes"]
    causes = json.load(open(causes_path)) if causes_path else {}
    print("| class | op | frac, box 0 / box 1 | kernel busy | dominant kernel, average launch | PMC / alg | launches "
          "| host / GPU ms per batch | below 0.70 |")
    print("|---|---|---|---|---|---|---|---|---|")
    for c, cv in a.items():
        if "error" in cv:
            print(f"| {c} | — | error: {cv['error']} | | | | | | |")
            continue
        for o in ("encode", "repair1", "repair2", "decode2"):
            x, y = cv.get(o), b.get(c, {}).get(o)
            if not isinstance(x, dict) or "frac" not in x:
                continue
            p, q = prof.get(c, {}).get(o, {}), pmc.get(c, {}).get(o, {})
            k = (p.get("dominant_kernel") or "").replace("gf_vec_kernel", "vec").replace(" ", "")
            low = x["frac"] < 0.70 or (y and y["frac"] < 0.70)
            cause = causes.get(f"{c}/{o}", "?") if low else "—"
            yb = f"{y['frac']:.3f}" if y else "—"
            print(f"| {c} | {o} | {x['frac']:.3f} / {yb} | {p.get('kernel_busy_frac')} | `{k}` {p.get('dominant_avg_us', 0):.0f} µs "
                  f"| {q.get('hbm_over_algorithmic')} | {x['launches_per_batch']:g} | {x['host_ms_per_batch']} / "
                  f"{x['ms_per_batch']} | {cause} |")


if len(sys.argv) > 1 and sys.argv[1] == "--markdown":
    markdown(*sys.argv[2:])
    sys.exit(0)

line = line_of(sys.argv[1])
prof = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else {"classes": {}}
for c, cv in line["classes"].items():
    if "error" in cv:
        print(c, cv["error"])
        continue
    ops = cv["ops"] if "ops" in cv else {o: v for o, v in cv.items() if isinstance(v, dict) and "frac" in v}
    for o, v in ops.items():
        p = prof["classes"].get(c, {}).get(o, {})
        print(f"{c:30s} {o:8s} S={cv['stripes_per_gpu']:4d} ms={v['ms_per_batch']:7.3f} frac={v['frac']:.3f} "
              f"exec/alg={v['executed_over_algorithmic']:.3f} launches={v['launches_per_batch']:5.1f} "
              f"calls={v.get('calls_per_batch')} host={v.get('host_ms_per_batch')} ok={v['verified']} | "
              f"{p.get('dominant_kernel')} avg={p.get('dominant_avg_us')}us busy={p.get('kernel_busy_frac')}")
