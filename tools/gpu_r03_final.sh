#!/bin/bash
# Round 3 end-of-round pass on the final tree.  Part a: GPU parity suite, smoke, default bench line,
# rocprofv3 kernel stats of the default line and of the headline alone (--no-config5 --no-ring
# --no-host-path, so the dominant kernel's average is the headline encode's), FETCH/WRITE PMC passes,
# N=1/N=2 rehearsal.  Part b (PART=b): every other workload, then rocprofv3 kernel stats of each.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
if [ "${PART:-a}" = "a" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -10; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 python bench.py > $O/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 40 --warmup 3 --no-cpu-baseline > "$R/$O/prof.log" 2>&1
  rc=$?; echo "rocprof default rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_headline" -o run --output-format csv -- python3 "$R/bench.py" --steps 40 --warmup 3 --no-cpu-baseline --no-config5 --no-ring --no-host-path > "$R/$O/prof_headline.log" 2>&1
  rc=$?; echo "rocprof headline rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/pmc_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-config5 --no-ring --no-host-path > "$R/$O/pmc_fetch.log" 2>&1
  rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/pmc_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-config5 --no-ring --no-host-path > "$R/$O/pmc_write.log" 2>&1
  rc=$?; echo "rocprof write rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$R" && python tools/parse_pmc.py "$O/pmc_fetch/**/*counter_collection.csv" "$O/pmc_write/**/*counter_collection.csv" $O/pmc_traffic.json rs104_B1048576_S4096 > /dev/null && echo pmc ok || exit 1
  bash tools/gpu_dist_rehearsal.sh > $O/rehearsal.log 2>&1
  rc=$?; echo "rehearsal rc=$rc"; tail -3 $O/rehearsal.log; exit $rc
else
  for w in rs-decode-patterns lrc-repair pc-merge rs4m-waves rs-host; do
    timeout -k 10 500 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.log 2>&1
    rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  for w in lrc-repair-ring lrc-global-ring pc-merge-ring; do
    timeout -k 10 300 python bench.py --workload $w --self-p2p > $O/bench_$w.log 2>&1
    rc=$?; echo "bench $w --self-p2p rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  cd /tmp && export TMPDIR=/tmp
  for w in rs-decode-patterns lrc-repair pc-merge rs4m-waves; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/wprof/$w" -o run --output-format csv -- \
      python3 "$R/bench.py" --workload $w --no-cpu-baseline > "$R/$O/wprof_$w.log" 2>&1
    rc=$?; echo "rocprof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
