"""One ECG_OPT_* option A/B'd inside one process on the same buffers: bench.py's own workload runs as usual,
but every timed step sets the option to the next value in rotation (forward / backward order on alternate
rounds), ROUNDS steps per value; per value the mean and best HIP-event time of the step (encode and decode
separately for the headline step) as a fraction of 8 TB/s.  Every form still verifies its outputs (bench).
usage: python opt_probe.py WORKLOAD FORMS OPTION ROUNDS V1 V2 ...   (FORMS "-" for none)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
workload, forms, option, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
values = [int(v) for v in sys.argv[5:]]
nv = len(values)
argv = [sys.argv[0], "--workload", workload, "--steps", str(nv * rounds), "--warmup", "2", "--no-cpu-baseline"]
if forms != "-":
    argv += ["--forms", forms]
sys.argv = argv
import bench  # noqa: E402
import ecg  # noqa: E402
import torch  # noqa: E402

per_form = []


def timed_loop(r, steps, step):
    evs = bench.events(steps)
    times = {v: [] for v in values}
    saved = ecg.get_option(option)
    try:
        for i in range(steps):
            rnd, j = divmod(i, nv)
            v = values[j] if rnd % 2 == 0 else values[nv - 1 - j]
            ecg.set_option(option, v)
            torch.cuda.synchronize()
            step(evs[i])
            torch.cuda.synchronize()
            e = evs[i]
            npairs = 2 if workload == "rs-encode-decode" else 1  # encode, decode / the whole step
            times[v].append([e[q].elapsed_time(e[q + 1]) for q in range(npairs)])
    finally:
        ecg.set_option(option, saved)
    per_form.append(times)
    return 1.0, evs


bench.timed_loop = timed_loop
a = bench.parse()
r = bench.D.Rank(0, 1, 0)
if workload == "rs-encode-decode":
    bench.rs_encode_decode(a, r)
    S, B = 4096, 1 << 20
    parts = [("encode", S * 14 * B), ("decode", S * 11 * B)]
    names = ["headline"]
else:
    fn = {"lrc-repair": bench.lrc_repair, "pc-merge": bench.pc_merge}[workload]
    res = fn(a, r)
    names = list(res["results"].keys())
    parts = [("step", res["algorithmic_bytes_per_batch"])]
out = {}
for name, times in zip(names, per_form):
    out[name] = {}
    for v, ts in times.items():
        d = {}
        for q, (pname, alg) in enumerate(parts):
            xs = [t[q] for t in ts]
            d[pname + "_frac_mean"] = round(alg / (sum(xs) / len(xs) / 1e3) / 8e12, 4)
            d[pname + "_frac_best"] = round(alg / (min(xs) / 1e3) / 8e12, 4)
        out[name][str(v)] = d
print(json.dumps({"workload": workload, "option": option, "results": out}))
