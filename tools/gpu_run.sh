#!/bin/bash
# One parameterised GPU-box runner (replaces the per-round tools/gpu_r0N_*.sh scripts).
#   OUT=<dir under gpurun_out/> bash tools/gpu_run.sh STEP [STEP ...]
# Steps, each under its own time limit; the run stops at the first step that fails:
#   tests      GPU parity suite (-m gpu, one process, per-test thread timeout)  -> pytest_gpu.log
#   test:<k>   GPU tests matching -k <k>                                          -> pytest_<k>.log
#   smoke      __graft_entry__.smoke()                                            -> smoke.log
#   bench      default bench line (python bench.py)                               -> bench.log
#   headline   bench line of the headline alone (no config 5 / ring / host path)  -> bench_headline.log
#   prof       rocprofv3 --kernel-trace --stats of the default line and of the headline alone
#   profh      the headline alone only (r06: the default line under rocprofv3 once died in the HIP runtime,
#              SIGSEGV inside hipLaunchKernel, during config 3's 8-thread per-call form)
#   pmc        FETCH_SIZE and WRITE_SIZE passes of the headline -> pmc_traffic.json (tools/parse_pmc.py)
#   summary    tools/profile_summary.py over prof_headline's trace + pmc_traffic.json -> headline_profile.json
#              (copy it and pmc_traffic.json to profiles/ to have bench.py's roofline name them)
#   rehearsal  bench.py --gpus 2 on the one GPU (tools/gpu_dist_rehearsal.sh)
#   rehearsal8 bench.py --gpus 8 on the one GPU, scaled down (tools/gpu_dist_rehearsal8.sh + check_rehearsal_n.py)
#   workloads  every bench.py --workload line                                    -> bench_<w>.log
#   wprof      rocprofv3 kernel stats of each non-default workload
#   w:<name>   one workload line                                                  -> bench_<name>.log
#   wp:<name>  rocprofv3 kernel stats of one workload
#   families   bench.py --workload families (every code class: encode, repairs, decode)   -> families.log
#   famprof    rocprofv3 kernel trace of the families workload + tools/families_profile.py -> families_profile.json
#   fampmc     FETCH_SIZE / WRITE_SIZE passes of the families workload -> families_pmc.json (per row HBM bytes)
#   percall    config 4's per-call merge sequence under launch-option variants (tools/percall_probe.py), one
#              rocprofv3 kernel trace sliced per variant                           -> percall_summary.json
#   w34prof    rocprofv3 kernel traces of each form the line's config3 / config4 objects time (one run per
#              form) -> workload_profile.json (tools/workload_profile.py; copy it to profiles/ for bench.py)
#   ceiling    tools/movement_ceiling: the product kernel's own access path with the multiply removed, and its
#              rocprofv3 kernel stats                                             -> ceiling.txt, ceiling_prof/
#   abrepair   config 3's per-call forms (1 and 8 threads), the tree's libecg vs $AB_LIB (default lib/ab/libecg.so;
#              loaded through ECG_LIB), alternated over 3 rounds                  -> abrepair_<v>_<r>.log
#   callrate   tools/call_rate + tools/record_cost (device-tier per-call cost)     -> call_rate.txt, record_cost.txt
#   ab         per-call cost A/B: the tree's libecg vs erasure-codes-prototype_amd/lib/ab/ (a build of an earlier
#              commit), tools/call_rate device + tools/record_cost, alternated over 3 rounds -> ab_<v>_<r>.txt
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-run}
mkdir -p "$O"
# heartbeat under gpurun_out/ (steps such as the PMC passes print nothing for minutes)
( while sleep 30; do date +%T >> "$O/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PYT="python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread"
HEADLINE="--no-config5 --no-ring --no-host-path --no-configs34 --no-families"

run() {  # name limit log cmd...  (the command's output goes to log; the status line to this script's stdout)
  local name=$1 lim=$2 log=$3; shift 3
  timeout -k 10 "$lim" "$@" >> "$log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}

prof() {  # dir log args...
  local d=$1 log=$2; shift 2
  (cd /tmp && TMPDIR=/tmp timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/$O/$d" -o run --output-format csv \
     -- python3 "$R/bench.py" "$@" > "$R/$O/$log" 2>&1)
  local rc=$?
  echo "rocprof $d rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}

pmc() {  # counter tag
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc "$1" -d "$R/$O/pmc_$2" -o "$2" --output-format csv \
     -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $HEADLINE > "$R/$O/pmc_$2.log" 2>&1)
  local rc=$?
  echo "pmc $1 rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}

WORKLOADS="rs-decode-patterns lrc-repair pc-merge rs4m-waves rs-host"
RINGS="lrc-repair-ring lrc-global-ring pc-merge-ring"

for step in "$@"; do
  case $step in
    tests) timeout -k 10 1200 $PYT tests -q -m gpu > "$O/pytest_gpu.log" 2>&1; rc=$?
           grep -E "^(FAILED|ERROR)|passed|failed" "$O/pytest_gpu.log" | tail -8; echo "tests rc=$rc"
           [ $rc -eq 0 ] || exit $rc ;;
    test:*) k=${step#test:}; L="$O/pytest_${k// /_}.log"
           timeout -k 10 600 $PYT tests -v -s -m gpu -k "$k" > "$L" 2>&1; rc=$?
           tail -3 "$L"; echo "test $k rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    smoke) run smoke 300 "$O/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"; tail -1 "$O/smoke.log" ;;
    bench) run bench 500 "$O/bench.log" python bench.py; tail -1 "$O/bench.log" | cut -c1-400 ;;
    headline) run headline 400 "$O/bench_headline.log" python bench.py --no-cpu-baseline $HEADLINE
           tail -1 "$O/bench_headline.log" | cut -c1-400 ;;
    prof) prof prof prof.log --steps 40 --warmup 3 --no-cpu-baseline
          rm -f "$O/prof/run_kernel_trace.csv"  # 10^5 rows (config 3's per-call forms): the stats stay
          prof prof_headline prof_headline.log --steps 40 --warmup 3 --no-cpu-baseline $HEADLINE ;;
    profh) prof prof_headline prof_headline.log --steps 40 --warmup 3 --no-cpu-baseline $HEADLINE ;;
    pmc) pmc FETCH_SIZE fetch; pmc WRITE_SIZE write
         python tools/parse_pmc.py "$O/pmc_fetch/**/*counter_collection.csv" "$O/pmc_write/**/*counter_collection.csv" \
           "$O/pmc_traffic.json" rs104_B1048576_S4096 > /dev/null && echo "pmc parse ok" || exit 1 ;;
    summary) python tools/profile_summary.py "$O/prof_headline/run_kernel_trace.csv" "$O/pmc_traffic.json" \
               "$O/headline_profile.json" 40 > /dev/null && echo "summary ok" || exit 1 ;;
    rehearsal) run rehearsal 600 "$O/rehearsal.log" bash tools/gpu_dist_rehearsal.sh; tail -3 "$O/rehearsal.log" ;;
    rehearsal8) run rehearsal8 1200 "$O/rehearsal8.log" env OUT=${OUT:-run}/rehearsal8 bash tools/gpu_dist_rehearsal8.sh; tail -3 "$O/rehearsal8.log" ;;
    workloads) for w in $WORKLOADS; do
                 run "bench $w" 500 "$O/bench_$w.log" python bench.py --workload $w --no-cpu-baseline
               done
               for w in $RINGS; do
                 run "bench $w" 300 "$O/bench_$w.log" python bench.py --workload $w --self-p2p
               done ;;
    wprof) for w in rs-decode-patterns lrc-repair pc-merge rs4m-waves; do
             prof "wprof/$w" "wprof_$w.log" --workload $w --no-cpu-baseline
           done ;;
    w:*) w=${step#w:}; run "bench $w" 500 "$O/bench_$w.log" python bench.py --workload $w --no-cpu-baseline
         tail -1 "$O/bench_$w.log" | cut -c1-600 ;;
    wp:*) w=${step#wp:}; prof "wprof/$w" "wprof_$w.log" --workload $w --no-cpu-baseline ;;
    families) run families 900 "$O/families.log" python bench.py --workload families --steps ${FSTEPS:-5} --warmup 2 \
                ${FARGS:-}; tail -c 600 "$O/families.log"; echo ;;
    famprof) prof famprof famprof.log --workload families --steps ${FSTEPS:-5} --warmup 2 --no-cpu-baseline ${FARGS:-}
             python tools/families_profile.py "$O/famprof/run_kernel_trace.csv" "$O/famprof.log" \
               "$O/families_profile.json" > "$O/families_profile.log" 2>&1 && echo "families_profile ok" || exit 1
             rm -f "$O/famprof/run_kernel_trace.csv" ;;  # summarised above; keeps gpurun_out under its copy-back cap
    percall) (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace -d "$R/$O/percall" -o run \
               --output-format csv -- python3 "$R/tools/percall_probe.py" run > "$R/$O/percall.log" 2>&1)
             rc=$?; echo "percall rc=$rc"; [ $rc -eq 0 ] || exit $rc
             python tools/percall_probe.py parse "$O/percall/run_kernel_trace.csv" "$O/percall.log" \
               > "$O/percall_summary.json" 2>&1 && echo "percall summary ok" || exit 1
             rm -f "$O/percall/run_kernel_trace.csv" ;;
    fampmc) for c in FETCH_SIZE WRITE_SIZE; do
              (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $c -d "$R/$O/fampmc_$c" -o run --output-format csv \
                 -- python3 "$R/bench.py" --workload families --steps 2 --warmup 1 --no-cpu-baseline ${FARGS:-} \
                 > "$R/$O/fampmc_$c.log" 2>&1); rc=$?; echo "fampmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
            done
            python tools/families_pmc.py "$O/fampmc_FETCH_SIZE/**/*counter_collection.csv" "$O/fampmc_FETCH_SIZE.log" \
              "$O/fampmc_WRITE_SIZE/**/*counter_collection.csv" "$O/fampmc_WRITE_SIZE.log" "$O/families_pmc.json" \
              > "$O/families_pmc.log" 2>&1 && echo "families pmc ok" || exit 1
            rm -rf "$O/fampmc_FETCH_SIZE" "$O/fampmc_WRITE_SIZE" ;;
    percall_plain) run percall_plain 600 "$O/percall_plain.log" python tools/percall_probe.py run ;;
    w34prof) C3="fused reference_sequence_scope_scratch reference_sequence_per_call reference_sequence_per_call_threads8"
             C4="rows fused reference_sequence_scope_scratch reference_sequence_per_call"
             spec=""
             for f in $C3; do
               prof "w34/c3_$f" "w34_c3_$f.log" --workload lrc-repair --forms $f --steps 10 --warmup 2 --no-cpu-baseline
               spec="$spec config3/$f=$O/w34/c3_$f/run_kernel_trace.csv:$O/w34_c3_$f.log:$f"
             done
             for f in $C4; do
               prof "w34/c4_$f" "w34_c4_$f.log" --workload pc-merge --forms $f --steps 10 --warmup 2 --no-cpu-baseline
               spec="$spec config4/$f=$O/w34/c4_$f/run_kernel_trace.csv:$O/w34_c4_$f.log:$f"
             done
             python tools/workload_profile.py "$O/workload_profile.json" $spec > "$O/workload_profile.log" 2>&1 \
               && echo "workload_profile ok" || exit 1
             # the per-call forms' traces run to 10^5 rows each: summarised above, the kernel stats stay
             rm -f "$O"/w34/*/run_kernel_trace.csv ;;
    ceiling) run ceiling 200 "$O/ceiling.txt" ./tools/movement_ceiling 4 10
             (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/ceiling_prof" -o run \
                --output-format csv -- "$R/tools/movement_ceiling" 2 10 > "$R/$O/ceiling_prof.txt" 2>&1)
             rc=$?; echo "ceiling prof rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    abrepair) for r in 1 2 3; do
                for v in new prev; do
                  if [ $v = prev ]; then EL=${AB_LIB:-$R/erasure-codes-prototype_amd/lib/ab/libecg.so}; else EL=$R/erasure-codes-prototype_amd/lib/libecg.so; fi
                  run "lrc per-call $v $r" 300 "$O/abrepair_${v}_$r.log" env ECG_LIB=$EL python bench.py --workload lrc-repair \
                    --forms reference_sequence_per_call,reference_sequence_per_call_threads8 --steps 10 --warmup 2 --no-cpu-baseline
                done
              done
              for f in "$O"/abrepair_*.log; do
                tail -1 "$f" | python -c "import json,sys; d=json.loads(sys.stdin.read())['results']; print('$f', {k: v['algorithmic_frac'] for k, v in d.items()})"
              done ;;
    callrate) run call_rate 300 "$O/call_rate.txt" ./tools/call_rate
              run record_cost 300 "$O/record_cost.txt" ./tools/record_cost ;;
    ab) for r in 1 2 3; do
          for v in new prev; do
            if [ $v = prev ]; then LP=$R/erasure-codes-prototype_amd/lib/ab; else LP=$R/erasure-codes-prototype_amd/lib; fi
            run "call_rate $v $r" 200 "$O/ab_${v}_$r.txt" env LD_LIBRARY_PATH=$LP ./tools/call_rate 3 device
            run "record_cost $v $r" 200 "$O/ab_${v}_$r.txt" env LD_LIBRARY_PATH=$LP ./tools/record_cost
          done
        done
        grep -H -E "dev_matrix|record " "$O"/ab_*.txt | cut -c1-160 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
