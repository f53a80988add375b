#!/bin/bash
# First GPU pass: parity suite, smoke, one bench line, rocprofv3 kernel-trace summary.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat gpurun_out/smoke.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name '*stats*' | head
exit $rc
