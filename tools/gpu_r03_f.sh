#!/bin/bash
# Round 3: call worker after the uniform-exit change -- its tests, three worker soaks, the whole suite.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_worker.log 2>&1
rc=$?; echo "worker tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|^E " $O/pytest_worker.log | tail -12; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  ECG_SOAK_OPS=2000 timeout -k 10 600 python -u -m pytest tests/test_gpu_stress.py -q -p no:cacheprovider -k "mixed_tiers and 2000" --timeout 500 --timeout-method thread > $O/soak2000_$i.log 2>&1
  rc=$?; echo "soak $i rc=$rc"; grep -E "passed|failed" $O/soak2000_$i.log | tail -1; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 env ECG_CALL_WORKER=2000 tools/small_call 4000 > $O/small_call_worker.log 2>&1; rc=$?; echo "small_call worker rc=$rc"; grep -E "^(call|callD|decD) " $O/small_call_worker.log
