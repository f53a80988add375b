#!/bin/bash
# Round 3, first GPU pass: parity suite, smoke, default bench line (with config5 + per-rank fractions),
# lrc-repair workload (reference sequence forms), N=2 shared-GPU rehearsal, rocprofv3 kernel stats of the
# default line, FETCH/WRITE PMC passes (headline only).
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=${O:-gpurun_out/r03a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload lrc-repair --steps 5 --warmup 2 > $O/bench_lrc-repair.log 2>&1
rc=$?; echo "lrc rc=$rc"; tail -1 $O/bench_lrc-repair.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_dist_rehearsal.sh > $O/rehearsal.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; tail -12 $O/rehearsal.log; cp -r gpurun_out/dist $O/dist 2>/dev/null; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 40 --warmup 3 --no-cpu-baseline > "$R/$O/prof.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_lrc" -o run --output-format csv -- python3 "$R/bench.py" --workload lrc-repair --steps 5 --warmup 2 > "$R/$O/prof_lrc.log" 2>&1
rc=$?; echo "rocprof lrc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/pmc_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-config5 > "$R/$O/pmc_fetch.log" 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/pmc_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-config5 > "$R/$O/pmc_write.log" 2>&1
rc=$?; echo "rocprof write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python tools/parse_pmc.py "$O/pmc_fetch/**/*counter_collection.csv" "$O/pmc_write/**/*counter_collection.csv" $O/pmc_traffic.json rs104_B1048576_S4096 > /dev/null && echo pmc ok
