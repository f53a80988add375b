// Completion flag of a latency-kernel workgroup, for a polling host (vector stores only).  A system-scope
// release is (1) the issuing wave's own stores complete (s_waitcnt vmcnt(0)), (2) the L2 written back
// (buffer_wbl2, which covers the whole L2, not one wave's lines) and (3) that write-back complete before
// the flag store.  So every wave waits for its own stores, the workgroup meets at a barrier, and only
// lane 0 of wave 0 writes the L2 back and posts the flag: one L2 write-back per workgroup instead of one
// per wave.  Step (3) is an explicit wait: after the barrier's vmcnt(0) the compiler's wait insertion
// does not count the write-back as outstanding and drops the wait a release store would carry (seen
// in the ISA: buffer_wbl2 directly followed by the flag store; a config-1 loopback run then read 3 of
// 2617 rebuilt blocks stale).  tests/test_flag_isa.py checks this sequence in the disassembly of every
// flag-posting kernel of libecg.so (tools/check_flag_isa.py).
//
// ECG_TEST_DROP_FLAG_WAIT removes the explicit wait of step (3).  It exists only so that the ISA check can
// be shown to catch the bug (tests/isa/flag_probe.hip; tools/build_variant.sh); never in a shipped build.
#pragma once

#include "gf_kernels.hpp"

namespace ecg {

// flag = this workgroup's slot (every thread of the workgroup calls this)
__device__ __forceinline__ void post_done_flag(unsigned* flag, unsigned seq) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0), expcnt / lgkmcnt unconstrained
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: buffer_wbl2
#ifndef ECG_TEST_DROP_FLAG_WAIT
        __builtin_amdgcn_s_waitcnt(0x0F70);            // the write-back has completed
#endif
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ void post_done_flag(const GfLaunch& a) {
    post_done_flag(a.done_flags + blockIdx.y * gridDim.x + blockIdx.x, a.done_seq);
}

}  // namespace ecg
