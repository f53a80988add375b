#!/bin/bash
# Round 3: cross-GPU partial decoding tests (local and global repairs, gloo N=2 shared GPU, RCCL self
# exchange) and the lrc-global-ring workload at N=1 (local helpers, --self-p2p) and N=2 (shared GPU).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gring
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -10; [ $rc -eq 0 ] || exit $rc
for m in "" "--self-p2p"; do
  timeout -k 10 200 python bench.py --workload lrc-global-ring $m --steps 5 --warmup 2 > $O/b$m.log 2>&1 || exit $?
  tail -1 $O/b$m.log
done
ECG_BENCH_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --workload lrc-global-ring --stripes 64 --chunk 16 \
  --steps 2 --warmup 1 > $O/n2.log 2>&1
rc=$?; grep "^{" $O/n2.log | tail -1; exit $rc
