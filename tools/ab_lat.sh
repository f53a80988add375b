#!/bin/bash
# A/B of two libecg builds on the latency paths: the tree's lib/ vs lib/ab/ (a build of the previous
# commit), small-call probe and per-stripe device calls, alternated over two rounds in one box.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/ab/pytest_gpu.log | tail -5; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
 for v in new prev; do
  if [ $v = prev ]; then export LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/erasure-codes-prototype_amd/lib/ab; else unset LD_LIBRARY_PATH; fi
  echo "== $v"
  timeout -k 10 120 tools/small_call 3000 > gpurun_out/ab/sc_${v}_$r.log 2>&1 || exit 1
  grep -E "^(parF |parFcp|callD|decD)" gpurun_out/ab/sc_${v}_$r.log
  timeout -k 10 120 tools/call_rate 3 device > gpurun_out/ab/dev_${v}_$r.log 2>&1 || exit 1
  grep dev_matrix gpurun_out/ab/dev_${v}_$r.log | cut -c1-110
 done
done
