#!/bin/bash
# Round 3: config 4's merge across GPUs (pc-merge-ring): GPU ring tests, the workload at N=1 (local,
# --self-p2p) and N=2 on the shared GPU.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pcring
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
for m in "" "--self-p2p"; do
  timeout -k 10 200 python bench.py --workload pc-merge-ring $m --steps 5 --warmup 2 > $O/b$m.log 2>&1 || exit $?
  tail -1 $O/b$m.log
done
ECG_BENCH_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --workload pc-merge-ring --stripes 16 --chunk 4 \
  --steps 2 --warmup 1 > $O/n2.log 2>&1
rc=$?; grep "^{" $O/n2.log | tail -1; exit $rc
