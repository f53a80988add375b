#!/bin/bash
# Round 3: the resident call worker -- its GPU tests, then the whole suite, then small-call timings.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_worker.log 2>&1
rc=$?; echo "worker tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Timeout" $O/pytest_worker.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 env ECG_CALL_WORKER=2000 tools/small_call 4000 > $O/small_call_worker.log 2>&1; rc=$?; echo "small_call worker rc=$rc"; head -3 $O/small_call_worker.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/small_call 4000 > $O/small_call_launch.log 2>&1; rc=$?; echo "small_call launch rc=$rc"; head -3 $O/small_call_launch.log
