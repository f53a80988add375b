#!/bin/bash
# Workgroup-size variants of libecg (tuning only): quick microbench per build, one process each.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in libecg libecg_tpb128 libecg_tpb64; do
  ECG_LIB=$GRAFT_REPO_ROOT/erasure-codes-prototype_amd/lib/$v.so timeout -k 10 300 python tools/microbench.py --quick --out gpurun_out/micro_$v.json > gpurun_out/micro_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_$v.log
  [ $rc -eq 0 ] || exit $rc
done
