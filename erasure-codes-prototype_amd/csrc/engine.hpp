// GF(2^8) region engine: turns LinearOps (matrix.hpp) into HIP launches on gfx950.
//
// Four ways in (plus run_host_pipeline for host-resident batches):
//   run_device  - block pointers are device pointers (HBM-resident), asynchronous on a stream;
//   run_host    - block pointers are host buffers (the reference's char** of host memory): blocks are
//                 staged into the device scratch of a pooled host context leased for the call, each
//                 block copied in at most once and every written block copied back once, then the
//                 stream is synchronised; small calls gather through a pinned staging area so a call
//                 costs one H2D and one D2H transfer;
//   run_strided - batches of S stripes laid out as base + stripe/block strides, each stripe running
//                 one of a small set of programs (e.g. 14 rotating single-erasure decode patterns).
// Coefficient tables are built on the host once per distinct program set and cached in HBM.
// Thread-safe: the cache is mutex-protected; host-tier scratch and streams belong to pooled contexts,
// one leased per call in flight.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ecg.h"  // status codes ECG_*
#include "gf_kernels.hpp"
#include "matrix.hpp"

namespace ecg {

// run_host staging thresholds: calls with blocks up to 256 KiB and at most 8 MiB of scratch go
// through the pinned staging area (memcpy + one DMA each way); larger ones copy block by block.
constexpr size_t kStagedMaxBlock = 256 << 10;
constexpr size_t kStagedMaxBytes = 8 << 20;

struct ProgramSet {
    CoefTab* d_tabs = nullptr;
    int* d_src = nullptr;
    int* d_dst = nullptr;
    int nprog = 0, k = 0, m = 0, MT = 1, rtiles = 1;
    bool binary = false;
    ~ProgramSet();
};

class Engine {
public:
    static Engine& instance();  // engine of the calling thread's current HIP device

    int run_device(const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B,
                   hipStream_t stream);
    int run_host(const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B);
    int run_strided(const std::vector<LinearOp>& progs, const int* d_prog_of_stripe, int S,
                    const void* in_base, long long in_sstride, long long in_bstride, void* out_base,
                    long long out_sstride, long long out_bstride, long long B, hipStream_t stream,
                    const int* d_stripe_of = nullptr);
    int run_ptrs(const LinearOp& prog, const uint8_t* const* d_src, uint8_t* const* d_dst, int S, long long B,
                 bool aligned16, hipStream_t stream);
    // One op over S calls' block pointers (host arrays): uploads the pointer tables, then run_ptrs.
    int run_ptr_batch(const LinearOp& op, const std::vector<const uint8_t* const*>& call_blocks, long long B,
                      hipStream_t stream);
    // The same, as ONE strided launch when the calls' blocks form base + call * sstride + id * bstride
    // (checked pointer by pointer); *done = false (nothing launched) otherwise.
    int run_calls_strided(const LinearOp& op, const std::vector<const uint8_t* const*>& calls, long long B,
                          hipStream_t stream, bool* done);

    // Host-resident batch (block b of stripe s at h_in + s*in_sstride + b*in_bstride, likewise out):
    // a 3-slot pipeline of H2D (2-D copies of the blocks the program reads), kernel, D2H (the blocks
    // it writes) on three streams, chunk_stripes stripes per slot.  Synchronous.
    int run_host_pipeline(const LinearOp& prog, const void* h_in, long long in_sstride, long long in_bstride,
                          void* h_out, long long out_sstride, long long out_bstride, long long B, int S,
                          int chunk_stripes);

    std::shared_ptr<ProgramSet> program_set(const std::vector<LinearOp>& progs, int* status);
    int host_contexts() const;  // host-tier contexts created so far (pooled; bounded by concurrent calls)
    int device() const { return device_; }
    size_t cache_size();

    int launch_direct(const std::vector<LinearOp>& ops, uint8_t* const* blocks, long long B, hipStream_t stream);

private:
    explicit Engine(int device);
    int launch_one(const LinearOp& op, uint8_t* const* blocks, long long B, hipStream_t stream);

    int device_;
    struct CacheEntry {
        std::shared_ptr<ProgramSet> ps;
        uint64_t last_use;
    };
    std::mutex mu_;
    uint64_t tick_ = 0;
    std::unordered_map<std::string, CacheEntry> cache_;  // LRU-bounded by ECG_OPT_PROGRAM_CACHE
};

// Deferred-batch scope of the calling thread (ecg_batch_begin / ecg_batch_end).  Inside a scope,
// device-tier calls (run_device: ecg_dev_matrix_*, ErasureCode objects on HBM buffers) are recorded
// instead of launched; batch_flush() launches each run of consecutive calls with the same plan and
// block size on the same stream as ONE launch per op -- strided when the run's blocks form one strided
// batch, a pointer-table launch otherwise -- splitting a run where a call touches a block an earlier
// call of the run writes (or writes one it reads).  Host-tier and batched calls flush first, so call
// order is kept.
int batch_begin();
int batch_flush();
int batch_end();
bool batch_active();

// Last HIP error seen by this thread (for diagnostics through the C ABI).
const char* last_error_string();
void set_last_error(const std::string& s);

}  // namespace ecg
