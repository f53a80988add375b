// Probe for tests/test_flag_isa.py: a kernel shaped like the latency kernels' tail (output stores, then the
// completion-flag epilogue of csrc/gf_done_flag.hpp), compiled device-only in seconds with and without
// ECG_TEST_DROP_FLAG_WAIT, to show that tools/check_flag_isa.py rejects the epilogue without its explicit
// wait.  Never launched.
#include "gf_done_flag.hpp"

__global__ void __launch_bounds__(256, 1) flag_probe_kernel(const ecg::GfLaunch a) {
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c < (a.B >> 2)) {
        const uint32_t x = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(a.isrc[0]) + c);
        __builtin_nontemporal_store(x ^ 0x5au, reinterpret_cast<uint32_t*>(a.idst[0]) + c);
    }
    if (a.done_flags) ecg::post_done_flag(a);
}
