#!/bin/bash
# Round 2, first GPU pass: new parity tests, the default bench line, the --gpus 2 launcher on a shared GPU.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "config5 or batch_scope_then or flush_on_recording" > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest new rc=$rc"; grep -E "PASS|FAIL|ERROR|SKIP" gpurun_out/pytest_new.log | tail -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
ECG_BENCH_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --stripes 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n2_shared.log 2>&1
rc=$?; echo "bench n2 shared rc=$rc"; tail -1 gpurun_out/bench_n2_shared.log; exit $rc
