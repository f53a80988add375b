#!/bin/bash
# Table-launch input grouping variants (tuning builds): kernel times of OFFS vs STRIDED per library.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ptrs3
O=$R/gpurun_out/ptrs3
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-libecg_fake libecg}; do
  ECG_LIB=$R/erasure-codes-prototype_amd/lib/$v.so timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$v -o run --output-format csv -- python3 $R/tools/mode_probe.py --reps 3 --cols 0 --tables ${TABLES:-1} > $O/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/$v.log; exit $rc; }
  python3 $R/tools/trace_summary.py "$O/$v/**/*kernel_trace.csv" gf_vec
done
