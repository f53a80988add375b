#!/bin/bash
# A/B of the BINARY 5-8-output occupancy hint (ECG_OCC_BIN_WIDE) on the pc-merge workload, rotated order.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03occ
mkdir -p $O
i=0
for v in libecg libecg_binocc6 libecg_binocc8 libecg libecg_binocc8 libecg_binocc6; do
  i=$((i+1))
  ECG_LIB=$GRAFT_REPO_ROOT/erasure-codes-prototype_amd/lib/$v.so timeout -k 10 200 python bench.py --workload pc-merge --steps 10 --warmup 3 > $O/pc_${i}_$v.log 2>&1
  rc=$?; echo "== $i $v rc=$rc"; tail -1 $O/pc_${i}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (v['ms_per_batch'], v['algorithmic_frac']) for k, v in d['results'].items()})"
  [ $rc -eq 0 ] || exit $rc
done
