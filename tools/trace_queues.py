"""Per-hardware-queue view of a rocprofv3 kernel trace: kernels, busy time, gaps between consecutive
kernels on a queue, and device-wide concurrency, over the last `--last` kernels whose name matches."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--match", default="gf_")
ap.add_argument("--last", type=int, default=0)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if a.match in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if a.last:
    rows = rows[-a.last:]
byq = collections.defaultdict(list)
for r in rows:
    byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
t0 = min(s for s, _ in (x for v in byq.values() for x in v))
t1 = max(e for _, e in (x for v in byq.values() for x in v))
print(f"{len(rows)} kernels over {(t1 - t0) / 1e3:.1f} us on {len(byq)} queues")
for q, v in sorted(byq.items()):
    busy = sum(e - s for s, e in v)
    gaps = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
    gaps.sort()
    med = gaps[len(gaps) // 2] if gaps else 0
    print(f"queue {q}: {len(v)} kernels, busy {busy / 1e3:.1f} us ({busy / (t1 - t0):.0%} of span), "
          f"avg kernel {busy / len(v) / 1e3:.2f} us, median gap {med / 1e3:.2f} us, mean gap "
          f"{sum(gaps) / max(1, len(gaps)) / 1e3:.2f} us")
ev = sorted([(s, 1) for v in byq.values() for s, _ in v] + [(e, -1) for v in byq.values() for _, e in v])
cur, prev, conc = 0, None, collections.Counter()
for t, d in ev:
    if prev is not None:
        conc[cur] += t - prev
    cur += d
    prev = t
tot = sum(conc.values())
print("concurrency (share of span):", {k: round(v / tot, 3) for k, v in sorted(conc.items())})
