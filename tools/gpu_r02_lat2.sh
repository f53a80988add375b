#!/bin/bash
# Round 2: latency kernel check -- GPU suite, the small-call probe, host-tier call latencies, then the
# small-call probe again under rocprofv3 --kernel-trace --stats (kernel durations vs the copy probes).
set -u
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/lat
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -8; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 tools/small_call 4000 > $O/small_call_$r.log 2>&1
  rc=$?; echo "small_call rc=$rc"; grep -E "^(empty|par|call|dec)" $O/small_call_$r.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  timeout -k 10 300 tools/call_rate 3 latency > $O/call_rate_latency_$r.log 2>&1
  rc=$?; echo "call_rate rc=$rc"; cat $O/call_rate_latency_$r.log; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $R/tools/small_call 2000 > $O/kt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
