#!/bin/bash
# Pointer-table launches (batch-scope flushes: config 3 / 4's per-call sequences in scopes with scratch) take grid
# map 1 under the auto rule.  A/B: the auto rule (ECG_GRID_MAP = 3) against map 2 forced for every launch
# (ECG_GRID_MAP = 2: stripe runs per XCD, the map the strided decode / repair / merge launches already take),
# interleaved over two rounds.  Speed only: every form verifies its outputs.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/ptrs_map; mkdir -p $O
for r in 1 2; do
  for gm in 3 2; do
    ECG_GRID_MAP=$gm timeout -k 10 300 python bench.py --workload lrc-repair --forms fused,reference_sequence_scope_scratch \
      --steps 10 --warmup 2 --no-cpu-baseline > $O/c3_r${r}_map$gm.log 2>&1 || exit 1
    ECG_GRID_MAP=$gm timeout -k 10 300 python bench.py --workload pc-merge --forms rows,reference_sequence_scope_scratch \
      --steps 10 --warmup 2 --no-cpu-baseline > $O/c4_r${r}_map$gm.log 2>&1 || exit 1
    for c in c3 c4; do
      python3 -c "import json; d=json.loads(open('$O/${c}_r${r}_map$gm.log').read().strip().splitlines()[-1]); print('$c', $r, 'map$gm', {k: v['algorithmic_frac'] for k, v in d['results'].items()})"
    done
  done
done
