#!/bin/bash
# Placement probe under rocprofv3: UTCL1 translation counters (pass a) and DRAM credit stalls + UTCL2 busy
# (pass b), one run each with the kernel trace; tools/parse_probe_pmc.py maps dispatches to variants.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ptlb; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_THRASHING_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum -d $O/a -o a --output-format csv -- python3 $R/tools/placement_probe.py --rounds 1 --reps 2 > $O/a.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_UTCL2_BUSY -d $O/b -o b --output-format csv -- python3 $R/tools/placement_probe.py --rounds 1 --reps 2 > $O/b.log 2>&1 || exit $?
ls -R $O | head; tail -n 12 $O/a.log $O/b.log
