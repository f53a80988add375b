#!/bin/bash
# Round 3: the default line at N = 5 on one shared GPU (gloo; timings meaningless): every rank's global-parity
# helpers at shifts 1..4 are four distinct peers, as on an 8-GPU node.  Sizes scaled down to fit five ranks.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/n5
mkdir -p $O
ECG_BENCH_SHARED_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 5 \
  --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 5 --stripes 64 --steps 2 --warmup 1 --no-cpu-baseline \
  --config5-stripes 2560 --config5-block-size 1048576 --ring-scale 0.0625 > $O/default_n5.log 2>&1
rc=$?; echo "rc=$rc"
grep "^{" $O/default_n5.log | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('n_gpus', d['n_gpus'], 'per_rank', len(d['per_rank']['encode_frac']))
ok = d['n_gpus'] == 5
for k in ('config5', 'host_path', 'ring_repair', 'global_ring_repair', 'merge_ring'):
    x = d[k]; v = x.get('verified_all_ranks', x.get('parity_checksum') is not None)
    print(k, v, x.get('error'), x.get('partials_over_rccl_per_repair', ''))
    ok &= bool(v) and 'error' not in x
print('N5', 'OK' if ok else 'MISMATCH'); sys.exit(0 if ok else 1)
" || exit 1
exit $rc
