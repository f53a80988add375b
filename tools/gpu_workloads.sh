#!/bin/bash
# GPU parity + every bench workload (single GPU).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_gpu.log | tail -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in ${WORKLOADS:-rs-encode-decode rs-decode-patterns lrc-repair lrc-repair-ring pc-merge rs4m-waves rs-host}; do
  timeout -k 10 500 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_$w.log | tail -3
  [ $rc -eq 0 ] || exit $rc
done
