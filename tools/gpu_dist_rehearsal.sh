#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2 ranks share cuda:0 (ECG_BENCH_SHARED_GPU=1, gloo for
# the bookkeeping collectives).  Checks that the sharded parity checksums combine to the N=1 value.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dist
O=gpurun_out/dist
run1() { timeout -k 10 300 python bench.py "$@" --steps 2 --warmup 1 --no-cpu-baseline; }
run2() { ECG_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
           --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 "$@" --steps 2 --warmup 1 --no-cpu-baseline; }
# default line incl. its config5 object: the full 65536 x 4 MiB batch at N = 1 and N = 2 (checksum == N = 1's)
run1 --stripes 512 > $O/rs_n1.log 2>&1 && echo "rs n1 ok" &&
run2 --stripes 256 > $O/rs_n2.log 2>&1 && echo "rs n2 ok" &&
ECG_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --stripes 256 --steps 2 --warmup 1 --no-cpu-baseline \
  --config5-stripes 2048 --config5-block-size 1048576 --timeout 380 \
  > $O/rs_n2_selfspawn.log 2>&1 && grep -q '"n_gpus": 2' $O/rs_n2_selfspawn.log && echo "rs n2 self-spawned ok" &&
run1 --workload rs4m-waves --stripes 2048 --block-size 1048576 > $O/waves_n1.log 2>&1 && echo "waves n1 ok" &&
run2 --workload rs4m-waves --stripes 2048 --block-size 1048576 > $O/waves_n2.log 2>&1 && echo "waves n2 ok" &&
run2 --workload lrc-repair --stripes 256 > $O/lrc_n2.log 2>&1 && echo "lrc n2 ok" &&
run2 --workload pc-merge --stripes 64 > $O/pc_n2.log 2>&1 && echo "pc n2 ok" &&
run2 --workload lrc-repair-ring --stripes 128 --chunk 32 > $O/ring_n2.log 2>&1 && echo "ring n2 ok" &&
python tools/check_dist_rehearsal.py $O
rc=$?
[ $rc -eq 0 ] || { for f in $O/*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -8; done; }
exit $rc
