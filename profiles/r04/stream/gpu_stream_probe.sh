#!/bin/bash
# Caller-stream lifetime: the destroyed/reused-stream GPU test with a native backtrace
# helper, then tools/stream_lifetime_probe's cases, each its own process, against the HIP runtime torch
# loads (torch/lib) and /opt/rocm's.  Stops at the first case that does not exit 0.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r04/stream}
mkdir -p $O
if [ "${SKIP_TEST:-0}" = "0" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_stress.py -x -v -s -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k destroyed > $O/test.log 2>&1
  rc=$?; echo "test rc=$rc"; tail -5 $O/test.log; [ $rc -eq 0 ] || exit $rc
fi
TORCH_LIB=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
for c in ${CASES:-8 4 1 3 6 5 2 7}; do
  for rt in torch rocm; do
    if [ $rt = torch ]; then LP=$TORCH_LIB; else LP=/opt/rocm/lib; fi
    LD_LIBRARY_PATH=$LP timeout -k 10 60 ./tools/stream_lifetime_probe $c > $O/case${c}_$rt.log 2>&1
    rc=$?; echo "case $c ($rt) rc=$rc"; cat $O/case${c}_$rt.log; [ $rc -eq 0 ] || exit $rc
  done
done
