#!/bin/bash
# GPU parity suite only (one process; per-test timeout interrupts a test stuck in a GPU call).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|Timeout" gpurun_out/pytest_gpu.log | tail -30
exit $rc
