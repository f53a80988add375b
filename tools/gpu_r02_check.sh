#!/bin/bash
# Round 2 check: full GPU suite, smoke, small-call probe, host-tier latencies, config-3 per-stripe forms.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/check
O=$R/gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/small_call 4000 > $O/small_call.log 2>&1
rc=$?; echo "small_call rc=$rc"; cat $O/small_call.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/call_rate 3 latency > $O/call_rate_latency.log 2>&1
rc=$?; echo "call_rate rc=$rc"; cat $O/call_rate_latency.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/scope_repair $((1<<20)) 4096 5 512 > $O/scope_repair.log 2>&1
rc=$?; echo "scope_repair rc=$rc"; cut -c1-140 $O/scope_repair.log; exit $rc
