#!/bin/bash
# lrc-repair's per-call reference sequence from 1/4/8/16 host threads: A/B of the
# device tier's latency-kernel threshold (ECG_LAT_DWORD_BYTES) and of the runtime's hardware queue count,
# then one rocprofv3 kernel trace of the 8-thread point.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r04/lrcmt}; mkdir -p $O
F=reference_sequence_per_call,reference_sequence_per_call_threads4,reference_sequence_per_call_threads8,reference_sequence_per_call_threads16
for lat in ${LATS:-1048576 262144 65536}; do
  for q in ${HWQS:-4}; do
    ECG_LAT_DWORD_BYTES=$lat GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --workload lrc-repair --no-cpu-baseline \
      --forms $F > $O/lat${lat}_hwq$q.log 2>&1 || exit 1
    echo "lat $lat hwq $q ok"
  done
done
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof8 -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --workload lrc-repair --no-cpu-baseline \
    --forms reference_sequence_per_call_threads8 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1 || exit 1
  echo prof ok
fi
if [ "${HIPTRACE:-0}" = "1" ]; then  # host-side HIP API durations under 1 and 8 issuing threads
  for f in reference_sequence_per_call reference_sequence_per_call_threads8; do
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --hip-trace --stats -d $GRAFT_REPO_ROOT/$O/hip_$f -o run \
      --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload lrc-repair --no-cpu-baseline \
      --forms $f --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/hip_$f.log 2>&1) || exit 1
    echo "hip trace $f ok"
  done
fi
