#!/bin/bash
# Round 3: N=2 shared-GPU rehearsal of the default line (config5 + per_rank + ring_repair), then the
# worker's prompt-exit test.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g
mkdir -p $O
bash tools/gpu_dist_rehearsal.sh > $O/rehearsal.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; tail -14 $O/rehearsal.log; cp -r gpurun_out/dist $O/dist 2>/dev/null; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_worker.py -v -p no:cacheprovider -k "exits_promptly" --timeout 120 --timeout-method thread > $O/exit_test.log 2>&1
rc=$?; echo "exit test rc=$rc"; grep -E "PASSED|FAILED|^E " $O/exit_test.log | head -5
