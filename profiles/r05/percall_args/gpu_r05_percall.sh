set -u
O=gpurun_out/r05_b; mkdir -p $O
PYT="python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests -v -s -m gpu -k "per_thread or eviction" > $O/pytest_per_thread.log 2>&1; rc=$?; tail -4 $O/pytest_per_thread.log; echo "per_thread rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in base lat256k lat256k_cpw256 lat256k_cpw512; do
  case $v in base) E="";; lat256k) E="ECG_LAT_DWORD_BYTES=262144";; lat256k_cpw256) E="ECG_LAT_DWORD_BYTES=262144 ECG_COLS_PER_WG=256";; lat256k_cpw512) E="ECG_LAT_DWORD_BYTES=262144 ECG_COLS_PER_WG=512";; esac
  for r in 1 2; do
    timeout -k 10 200 env $E python bench.py --workload lrc-repair --forms reference_sequence_per_call,reference_sequence_per_call_threads8 --steps 10 --warmup 2 --no-cpu-baseline > $O/pc_${v}_$r.log 2>&1 || exit 1
    tail -1 $O/pc_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read())['results']; print('$v $r', {k: v['algorithmic_frac'] for k, v in d.items()})"
  done
done
(cd /tmp && export TMPDIR=/tmp ECG_LAT_DWORD_BYTES=262144 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_vec -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload lrc-repair --forms reference_sequence_per_call --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_vec.log 2>&1) || exit 1
echo "--- expected to FAIL on the round-4 build (ECG_LIB=lib/ab):"
ECG_LIB=$GRAFT_REPO_ROOT/erasure-codes-prototype_amd/lib/ab/libecg.so timeout -k 10 300 $PYT tests -v -s -m gpu -k "per_thread" > $O/pytest_per_thread_r04build.log 2>&1; echo "r04 build per_thread rc=$?"; tail -5 $O/pytest_per_thread_r04build.log
