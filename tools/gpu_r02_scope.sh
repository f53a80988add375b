#!/bin/bash
# Round 2: batch-scope grouping + scratch composition -- GPU parity of the scope tests, then config 3's
# per-stripe partial-decoding sequence in four forms (tools/scope_repair) and its kernel stats.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/scope
O=$R/gpurun_out/scope
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -14; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 tools/scope_repair $((1<<20)) 4096 5 512 > $O/scope_repair.log 2>&1
rc=$?; echo "scope_repair rc=$rc"; cat $O/scope_repair.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $R/tools/scope_repair $((1<<20)) 4096 3 512 > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
head -12 $O/prof/run_kernel_stats.csv | cut -c1-200
