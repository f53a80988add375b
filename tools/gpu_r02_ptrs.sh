#!/bin/bash
# Pointer-table (PTRS) vs strided kernel on the config-2 batch: kernel times per COLS_PER_WG and SQ counters.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ptrs
O=$R/gpurun_out/ptrs
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/tools/mode_probe.py --reps 4 --cols 0,256,512,1024 > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/trace.log; exit $rc; }
python3 $R/tools/trace_summary.py "$O/trace/**/*kernel_trace.csv" gf_vec > $O/trace_summary.txt; cat $O/trace_summary.txt
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VALU -d $O/pmc_sq -o sq --output-format csv -- python3 $R/tools/mode_probe.py --reps 2 --cols 0 > $O/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/pmc_sq.log; exit $rc; }
ls -R $O/pmc_sq | head
