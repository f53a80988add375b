#!/bin/bash
# Round 2: table-launch parity, then OFFS vs PTRS vs STRIDED kernel times + SQ counters.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/ptrs2
O=$R/gpurun_out/ptrs2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "batch_scope" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/tools/mode_probe.py --reps 4 --cols 0 --tables 1,0 > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/trace.log; exit $rc; }
python3 $R/tools/trace_summary.py "$O/trace/**/*kernel_trace.csv" gf_vec > $O/trace_summary.txt; cat $O/trace_summary.txt
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VALU -d $O/pmc_sq -o sq --output-format csv -- python3 $R/tools/mode_probe.py --reps 2 --cols 0 --tables 1,0 > $O/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; exit $rc
