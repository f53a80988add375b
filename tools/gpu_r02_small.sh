#!/bin/bash
# Round 2: the small synchronous host-tier call (config 1's shape) against the launch + sync floor,
# plain and under rocprofv3 --kernel-trace --hip-trace --stats.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/small
O=$R/gpurun_out/small
timeout -k 10 120 $R/tools/small_call 4000 > $O/small_call.log 2>&1
rc=$?; echo "small_call rc=$rc"; cat $O/small_call.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --stats -d $O/trace -o run --output-format csv -- $R/tools/small_call 2000 > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/trace.log; exit $rc; }
cat $O/trace.log | tail -4
ls $O/trace
