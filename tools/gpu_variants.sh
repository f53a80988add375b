#!/bin/bash
# Workgroup-size variants of libecg (tuning only): quick microbench per build, one process each, run in
# rotated order twice so process-order effects are visible.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for v in ${VARIANTS:-libecg_tpb256 libecg libecg_tpb64 libecg libecg_tpb256}; do
  i=$((i+1))
  ECG_LIB=$GRAFT_REPO_ROOT/erasure-codes-prototype_amd/lib/$v.so timeout -k 10 300 python tools/microbench.py --quick --out gpurun_out/micro_${i}_$v.json > gpurun_out/micro_${i}_$v.log 2>&1
  rc=$?; echo "== $i $v rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_${i}_$v.log
  [ $rc -eq 0 ] || exit $rc
done
