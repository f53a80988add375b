#!/bin/bash
# Round 3: the whole GPU suite under non-default engine options (results must never depend on them):
# the resident call worker on for every eligible host call; DMA staging instead of zero-copy with the
# 16-bytes-per-lane kernel for single calls; the stripe-per-XCD grid map everywhere.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/optenv
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/$tag.log 2>&1; local rc=$?; echo "$tag: $(grep -E 'passed|failed' $O/$tag.log | tail -1)"; grep -E "^FAILED" $O/$tag.log | head -5; return $rc; }
run worker ECG_CALL_WORKER=500 && run dma16 ECG_ZEROCOPY_BYTES=0 ECG_LAT_DWORD_BYTES=0 && run map2 ECG_GRID_MAP=2
