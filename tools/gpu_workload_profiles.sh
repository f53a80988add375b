#!/bin/bash
# rocprofv3 --kernel-trace --stats of every non-default bench workload (one pass each, no counters).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p "$R/gpurun_out/wprof"
cd /tmp && export TMPDIR=/tmp
for w in ${WORKLOADS:-rs-decode-patterns lrc-repair lrc-repair-ring pc-merge rs4m-waves}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/wprof/$w" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload $w --no-cpu-baseline > "$R/gpurun_out/wprof/$w.log" 2>&1
  rc=$?; echo "rocprof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
