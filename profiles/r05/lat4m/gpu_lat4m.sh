#!/bin/bash
# Config 4's per-call sequence (4 MiB calls) on the vector kernel (default: ECG_LAT_DWORD_BYTES = 1 MiB) against
# the 4-byte-lane latency kernel (ECG_LAT_DWORD_BYTES = 4 MiB), interleaved, then one rocprofv3 stats run each.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/lat4m; mkdir -p $O
F="--workload pc-merge --forms reference_sequence_per_call,reference_sequence_scope --steps 10 --warmup 2 --no-cpu-baseline"
for r in 1 2; do
  for v in 1048576 4194304 2097152; do
    ECG_LAT_DWORD_BYTES=$v timeout -k 10 300 python bench.py $F > $O/run${r}_$v.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/run${r}_$v.log').read().strip().splitlines()[-1]); print($r, $v, {k: v['algorithmic_frac'] for k, v in d['results'].items()})"
  done
done
for v in 1048576 4194304; do
  (cd /tmp && TMPDIR=/tmp ECG_LAT_DWORD_BYTES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o run \
     --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload pc-merge --forms reference_sequence_per_call --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1) || exit 1
  head -3 $O/prof_$v/*kernel_stats.csv | cut -c1-200
  rm -f $O/prof_$v/*kernel_trace.csv
done
