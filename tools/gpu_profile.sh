#!/bin/bash
# Round profile: parity suite, bench line, rocprofv3 kernel-trace stats, two PMC passes (HBM bytes).
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_gpu.log | tail -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/microbench.py --out gpurun_out/micro.json > gpurun_out/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 40 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_fetch.log" 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_write.log" 2>&1
rc=$?; echo "rocprof write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python tools/parse_pmc.py "gpurun_out/pmc_fetch/**/*counter_collection.csv" "gpurun_out/pmc_write/**/*counter_collection.csv" gpurun_out/pmc_traffic.json rs104_B1048576_S4096
