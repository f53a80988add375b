#!/bin/bash
# Copy one final pass (tools/gpu_run.sh tests smoke headline prof|profh pmc summary w34prof famprof fampmc
# [bench rehearsal8] [ceiling], merged back under gpurun_out/) into profiles/rNN/NAME/, replacing what was there, and
# point the committed summaries bench.py reads (profiles/headline_profile.json, pmc_traffic.json,
# workload_profile.json, families_profile.json) at the copies.  Steps a pass did not run are skipped.
#   tools/collect_final.sh gpurun_out/r06/final4 profiles/r06/final
set -euo pipefail
cd "$(dirname "$0")/.."
S=$1; D=$2
rm -rf "$D"
mkdir -p "$D/workloads" "$D/families"
cpif() { [ -e "$1" ] && cp "$1" "$2" || true; }
for f in bench.log bench_headline.log pytest_gpu.log smoke.log pmc_traffic.json headline_profile.json; do cpif "$S/$f" "$D/"; done
cpif "$S/prof/run_kernel_stats.csv" "$D/rocprof_kernel_stats_bench_default_line.csv"
cp "$S/prof_headline/run_kernel_stats.csv" "$D/rocprof_kernel_stats_bench_headline.csv"
cp "$S/prof_headline/run_kernel_trace.csv" "$D/rocprof_kernel_trace_bench_headline.csv"
cp "$S/pmc_fetch/fetch_counter_collection.csv" "$D/pmc_fetch_counter_collection.csv"
cp "$S/pmc_write/write_counter_collection.csv" "$D/pmc_write_counter_collection.csv"
for f in "$S"/w34_c*.log; do b=$(basename "$f"); cp "$f" "$D/workloads/bench_${b#w34_}"; done
for d in "$S"/w34/*/; do n=$(basename "$d"); cp "$d/run_kernel_stats.csv" "$D/workloads/rocprof_kernel_stats_$n.csv"; done
cp "$S/families_profile.json" "$S/families_pmc.json" "$S/famprof.log" "$D/families/"
cp "$S/famprof/run_kernel_stats.csv" "$D/families/rocprof_kernel_stats_families.csv"
if [ -d "$S/rehearsal8" ]; then
  mkdir -p "$D/rehearsal8"; cp "$S"/rehearsal8/*.log "$D/rehearsal8/" 2>/dev/null || true
  cpif "$S/rehearsal8.log" "$D/rehearsal8/check.log"
fi
if [ -e "$S/ceiling.txt" ]; then
  mkdir -p "$D/ceiling"; cp "$S/ceiling.txt" "$S/ceiling_prof.txt" "$D/ceiling/"
  cp "$S"/ceiling_prof/*kernel_stats.csv "$D/ceiling/rocprof_kernel_stats_ceiling.csv"
fi
python3 - "$S" "$D" <<'PY'
import json, sys
S, D = sys.argv[1], sys.argv[2]
h = json.load(open(f"{D}/headline_profile.json"))
h["source"], h["pmc_source"] = f"{D}/rocprof_kernel_trace_bench_headline.csv", f"{D}/pmc_traffic.json"
p = json.load(open(f"{D}/pmc_traffic.json"))
for k, v in list(p.items()):
    if isinstance(v, str) and S in v:
        p[k] = (v.replace(f"{S}/pmc_fetch/fetch_counter_collection.csv", f"{D}/pmc_fetch_counter_collection.csv")
                 .replace(f"{S}/pmc_write/write_counter_collection.csv", f"{D}/pmc_write_counter_collection.csv")
                 .replace(S, D))
w = json.load(open(f"{S}/workload_profile.json"))
for k, v in w["forms"].items():
    cfg, form = k.split("/")
    wl = "lrc-repair" if cfg == "config3" else "pc-merge"
    v["source"] = (f"rocprofv3 --kernel-trace of bench.py --workload {wl} --forms {form} --steps 10 --warmup 2 "
                   f"(trace summarised on the box, not kept; {D}/workloads/)")
    for kk in ("kernel_stats", "bench_log"):
        if kk in v:
            v[kk] = (v[kk].replace(f"{S}/w34_", f"{D}/workloads/bench_").replace(f"{S}/w34/", f"{D}/workloads/rocprof_kernel_stats_")
                     .replace("/run_kernel_stats.csv", ".csv"))
f = json.load(open(f"{D}/families/families_profile.json"))
for obj, paths in ((h, (f"{D}/headline_profile.json", "profiles/headline_profile.json")),
                   (p, (f"{D}/pmc_traffic.json", "profiles/pmc_traffic.json")),
                   (w, (f"{D}/workloads/workload_profile.json", "profiles/workload_profile.json")),
                   (f, ("profiles/families_profile.json",))):
    for path in paths:
        json.dump(obj, open(path, "w"), indent=1)
print("libecg", h["libecg_sha16"], p.get("libecg_sha16"), w["libecg_sha16"], f.get("libecg_sha16"))
PY
