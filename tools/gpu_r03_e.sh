#!/bin/bash
# Round 3: every bench workload + their rocprofv3 kernel stats, and an 8-thread x 2000-operation soak with
# the resident call worker on.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=gpurun_out/r03e
mkdir -p $O
ECG_SOAK_OPS=2000 timeout -k 10 600 python -u -m pytest tests/test_gpu_stress.py -q -p no:cacheprovider -k "mixed_tiers" --timeout 500 --timeout-method thread > $O/soak2000.log 2>&1
rc=$?; echo "soak rc=$rc"; grep -E "passed|failed" $O/soak2000.log | tail -2; [ $rc -eq 0 ] || exit $rc
for w in rs-decode-patterns lrc-repair lrc-repair-ring pc-merge rs4m-waves rs-host; do
  timeout -k 10 500 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; grep -v amdgpu.ids $O/bench_$w.log | tail -1 | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
for w in rs-decode-patterns pc-merge rs4m-waves; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/wprof/$w" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload $w --no-cpu-baseline > "$R/$O/wprof_$w.log" 2>&1
  rc=$?; echo "rocprof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
