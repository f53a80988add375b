"""Grid map of pointer-table launches, A/B inside one process (same buffers, same physical pages): bench.py's
config-3 / config-4 forms run as usual, but every timed step alternates ECG_OPT_GRID_MAP between the auto
rule (3: pointer tables take map 1) and map 2 (stripe runs per XCD), several rounds; per map the mean and
min of the step's HIP-event time and its algorithmic fraction.  Every form still verifies its outputs (bench).
usage: python ptrs_map_probe.py lrc-repair|pc-merge FORMS ROUNDS"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
workload, forms, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3])
sys.argv = [sys.argv[0], "--workload", workload, "--forms", forms, "--steps", str(2 * rounds), "--warmup", "2",
            "--no-cpu-baseline"]
import bench  # noqa: E402
import ecg  # noqa: E402
import torch  # noqa: E402

MAPS = (3, 2)
per_form = {}
cur = {"form": None}


def timed_loop(r, steps, step):
    evs = bench.events(steps)
    times = {m: [] for m in MAPS}
    saved = ecg.get_option(ecg.ECG_OPT_GRID_MAP)
    try:
        for i in range(steps):
            m = MAPS[i % 2] if (i // 2) % 2 == 0 else MAPS[1 - i % 2]  # ABBA order
            ecg.set_option(ecg.ECG_OPT_GRID_MAP, m)
            torch.cuda.synchronize()
            step(evs[i])
            torch.cuda.synchronize()
            times[m].append(evs[i][0].elapsed_time(evs[i][1]))
    finally:
        ecg.set_option(ecg.ECG_OPT_GRID_MAP, saved)
    per_form.setdefault(len(per_form), times)
    return 1.0, evs


bench.timed_loop = timed_loop
a = bench.parse()
r = bench.D.Rank(0, 1, 0)
fn = bench.lrc_repair if workload == "lrc-repair" else bench.pc_merge
res = fn(a, r)
names = list(res["results"].keys())
alg = res["algorithmic_bytes_per_batch"]
out = {}
for i, name in enumerate(names):
    t = per_form[i]
    out[name] = {f"map{m}": {"mean_ms": round(sum(v) / len(v), 3), "min_ms": round(min(v), 3),
                             "frac_mean": round(alg / (sum(v) / len(v) / 1e3) / 8e12, 4),
                             "frac_best": round(alg / (min(v) / 1e3) / 8e12, 4), "n": len(v)} for m, v in t.items()}
print(json.dumps({"workload": workload, "results": out}))
