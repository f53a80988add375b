#!/bin/bash
# Round 3: batch-flush fast path (one overlap-free strided group without the hazard hash): the scope's GPU
# tests, the random-sequence and sliding-window checks, then per-stripe call rates in a scope.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fastpath
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stress.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "batch or concurrent" > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAIL" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 120 tools/call_rate 3 device > $O/call_rate_$r.log 2>&1 || exit $?; grep -E "batch scope" $O/call_rate_$r.log; done
