#!/bin/bash
# Rehearse the driver's SCALE command at N = 8 on a one-GPU box: `bench.py --gpus 8`
# starts its own 8 ranks, all on cuda:0 (ECG_BENCH_SHARED_GPU=1, gloo for the bookkeeping and the ring
# exchanges), with the default line scaled down to fit one GPU: 64 headline stripes per rank, ring objects
# at 1/8 size, config 5 at 2048 stripes of 4 MiB, configs 3 / 4 at 128 repairs / 16 merges per rank, the families at 0.5 GiB per class.  The N = 1 run covers the same global stripes (8 x 64);
# tools/check_rehearsal_n.py then checks every sub-object at world 8 against it.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r04/rehearsal8}
mkdir -p $O
N=${N:-8}
# heartbeat under gpurun_out/ while the ranks run (they print only their final line)
( while sleep 30; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
COMMON="--ring-scale 0.125 --config5-stripes 2048 --configs34-stripes 128 --working-set-gib 0.5 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 python bench.py --stripes $((64 * N)) $COMMON > $O/rs_n1.log 2>&1 && echo "rs n1 ok" &&
ECG_BENCH_SHARED_GPU=1 timeout -k 10 900 python bench.py --gpus $N --stripes 64 $COMMON --timeout 850 \
  > $O/rs_n$N.log 2>&1 && echo "rs n$N ok" &&
python tools/check_rehearsal_n.py $O/rs_n1.log $O/rs_n$N.log $N
rc=$?
[ $rc -eq 0 ] || { for f in $O/*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -8; done; }
exit $rc
