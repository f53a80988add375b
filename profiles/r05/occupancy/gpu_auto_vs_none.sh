#!/bin/bash
# The input-count pad table (ECG_OPT_MT1_LDS_PAD = -1, the default) against no pad (0), one process per
# workload on the same buffers (opt_probe.py, 6 rounds), after the new GPU test.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/occupancy/${TAG:-auto}; mkdir -p $O
P=profiles/r05/occupancy/opt_probe.py
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "mt1_lds_pad or tuning_options" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python $P rs-encode-decode - 10 6 -1 0 > $O/headline.log 2>&1 || exit 1
tail -1 $O/headline.log
timeout -k 10 300 python $P lrc-repair fused,reference_sequence_scope_scratch 10 6 -1 0 > $O/c3.log 2>&1 || exit 1
tail -1 $O/c3.log
timeout -k 10 300 python $P pc-merge rows,reference_sequence_scope_scratch,reference_sequence_per_call 10 6 -1 0 > $O/c4.log 2>&1 || exit 1
tail -1 $O/c4.log
