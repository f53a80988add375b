#!/bin/bash
# Round 3: call-worker validation -- GPU suite (incl. worker, soak and loopback variants), host-tier call
# rates with and without the worker, the persistent probe's queue-interference check.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/call_rate 3 latency > $O/call_rate_launch.log 2>&1; rc=$?; echo "call_rate launch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env ECG_CALL_WORKER=2000 tools/call_rate 3 latency > $O/call_rate_worker.log 2>&1; rc=$?; echo "call_rate worker rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 env ECG_CALL_WORKER=2000 tools/small_call 4000 > $O/small_call_worker.log 2>&1; rc=$?; echo "small_call worker rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/small_call 4000 > $O/small_call_launch.log 2>&1; rc=$?; echo "small_call launch rc=$rc"
grep -E "^(call|decD|callD) " $O/small_call_*.log
tail -20 $O/call_rate_worker.log
