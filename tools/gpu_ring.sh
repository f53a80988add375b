#!/bin/bash
# Cross-GPU partial decoding (lrc-repair-ring): GPU parity tests, the N=1 bench line at full size with a
# chunk sweep, and the 2-rank shared-GPU rehearsal (gloo; the N>1 rate needs an 8-GPU node).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ring
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > $O/pytest.log 2>&1 && echo "tests ok" &&
for c in 16 64 256; do
  timeout -k 10 300 python bench.py --workload lrc-repair-ring --chunk $c --steps 10 --warmup 2 > $O/n1_chunk$c.log 2>&1 || exit 1
  echo "n1 chunk $c ok"
done &&
ECG_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --workload lrc-repair-ring --stripes 256 --chunk 64 \
  --steps 2 --warmup 1 > $O/n2_shared.log 2>&1 && echo "n2 shared ok"
rc=$?
for f in $O/*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -3; done
exit $rc
