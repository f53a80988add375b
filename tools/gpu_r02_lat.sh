#!/bin/bash
# Round 2: the small-call latency kernel's lane width (4 vs 16 bytes per lane) -- GPU suite, small-call
# probe A/B, host-tier latencies with the default and with ECG_LAT_DWORD_BYTES=0 (16 bytes per lane).
set -u
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/lat
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/small_call 4000 > $O/small_call.log 2>&1
rc=$?; echo "small_call rc=$rc"; cat $O/small_call.log; [ $rc -eq 0 ] || exit $rc
for v in default 0 default 0; do
  if [ $v = default ]; then
    timeout -k 10 300 tools/call_rate 3 latency > $O/call_rate_latency_$v.log 2>&1
  else
    ECG_LAT_DWORD_BYTES=$v timeout -k 10 300 tools/call_rate 3 latency > $O/call_rate_latency_$v.log 2>&1
  fi
  rc=$?; echo "call_rate ($v) rc=$rc"; cat $O/call_rate_latency_$v.log; [ $rc -eq 0 ] || exit $rc
done
