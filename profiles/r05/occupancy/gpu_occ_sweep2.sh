#!/bin/bash
# Finer ECG_OPT_MT1_LDS_PAD sweep (option 10), one process per workload (opt_probe.py), 6 rounds.
# Pads as workgroups per CU at 160 KiB of LDS: 16384 = 10, 18176 = 9, 20480 = 8, 22528 = 7, 24576 = 6,
# 27136 = 6, 32768 = 5, 40960 = 4.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/occupancy/${TAG:-b2}; mkdir -p $O
P=profiles/r05/occupancy/opt_probe.py
timeout -k 10 300 python $P rs-encode-decode - 10 6 0 18176 20480 22528 24576 27136 32768 > $O/sweep_headline.log 2>&1 || exit 1
tail -1 $O/sweep_headline.log
timeout -k 10 300 python $P lrc-repair fused,reference_sequence_scope_scratch 10 6 0 16384 18176 20480 22528 24576 > $O/sweep_c3.log 2>&1 || exit 1
tail -1 $O/sweep_c3.log
timeout -k 10 300 python $P pc-merge rows,reference_sequence_scope_scratch 10 6 0 22528 24576 27136 32768 40960 > $O/sweep_c4.log 2>&1 || exit 1
tail -1 $O/sweep_c4.log
