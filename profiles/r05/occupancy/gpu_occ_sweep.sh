#!/bin/bash
# ECG_OPT_MT1_LDS_PAD (option 10) swept inside one process per workload (opt_probe.py).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/occupancy; mkdir -p $O
P=profiles/r05/occupancy/opt_probe.py
if [ "${SKIP_HEADLINE:-0}" = 0 ]; then
timeout -k 10 300 python $P rs-encode-decode - 10 4 0 12288 14336 16384 18432 20480 22528 24576 26624 > $O/sweep_headline.log 2>&1 || exit 1
tail -1 $O/sweep_headline.log
fi
timeout -k 10 300 python $P lrc-repair fused,reference_sequence_scope_scratch 10 4 0 16384 20480 22528 24576 > $O/sweep_c3.log 2>&1 || exit 1
tail -1 $O/sweep_c3.log
timeout -k 10 300 python $P pc-merge rows,reference_sequence_scope_scratch 10 4 0 16384 20480 22528 24576 > $O/sweep_c4.log 2>&1 || exit 1
tail -1 $O/sweep_c4.log
