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

#include <algorithm>
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
// A flush launches each run on its engine's device (the calling thread's device is restored after).  If a
// launch fails, the flush stops there and returns the error; the calls of that run and of every later
// run are dropped (not retried by a later flush).
int batch_begin();
int batch_flush();
int batch_end();
bool batch_active();
// Flush this thread's recorded calls, if any (entry points that launch directly call it first, so a
// recorded call never runs after a later direct launch).
int batch_flush_pending();

// Open-addressing set of block addresses for the flush's hazard check: a run of S recorded calls puts
// S * (k + m) addresses through it, and node-based hashing made that check most of a flush.  Addresses
// are never null (validated at record time), so 0 marks an empty slot.
class PtrSet {
public:
    void clear() {  // O(table): shrink a table a large run left behind before many small runs reuse it
        if (slots_.size() > 4096 && count_ * 8 < slots_.size()) {
            slots_.assign(1024, 0);
            mask_ = 1023;
        } else if (count_) {
            std::fill(slots_.begin(), slots_.end(), (uintptr_t)0);
        }
        count_ = 0;
    }
    bool contains(const void* ptr) const {
        if (slots_.empty()) return false;
        const uintptr_t p = (uintptr_t)ptr;
        for (size_t i = hash(p) & mask_;; i = (i + 1) & mask_) {
            if (slots_[i] == p) return true;
            if (slots_[i] == 0) return false;
        }
    }
    void insert(const void* ptr) {
        if ((count_ + 1) * 2 > slots_.size()) grow();
        const uintptr_t p = (uintptr_t)ptr;
        for (size_t i = hash(p) & mask_;; i = (i + 1) & mask_) {
            if (slots_[i] == p) return;
            if (slots_[i] == 0) {
                slots_[i] = p;
                count_++;
                return;
            }
        }
    }
    size_t size() const { return count_; }

private:
    static size_t hash(uintptr_t p) { return (size_t)(((unsigned long long)p >> 4) * 0x9E3779B97F4A7C15ull >> 17); }
    void grow() {
        std::vector<uintptr_t> old;
        old.swap(slots_);
        slots_.assign(old.empty() ? 1024 : old.size() * 2, 0);
        mask_ = slots_.size() - 1;
        count_ = 0;
        for (uintptr_t p : old)
            if (p) insert((const void*)p);
    }
    std::vector<uintptr_t> slots_;
    size_t mask_ = 0, count_ = 0;
};

// Run formation of the flush (pure host logic, no HIP; fuzzed against a quadratic check in
// tests/sanitize/host_fuzz.cpp).  Splits calls [0, n) into maximal runs [i, j): every call of a run has
// same_run(i, c) true, and no call reads or writes a block an earlier call of its run writes, or writes a
// block an earlier call of its run reads.  reads(c, f) / writes(c, f) call f(address) for each block call
// c reads / writes.  Returns the run ends (the last one is n).
template <class SameRun, class Reads, class Writes>
std::vector<size_t> form_runs(size_t n, SameRun same_run, Reads reads, Writes writes) {
    std::vector<size_t> ends;
    PtrSet wr, rd;
    size_t i = 0;
    while (i < n) {
        wr.clear();
        rd.clear();
        auto add = [&](size_t c) {
            reads(c, [&](const void* p) { rd.insert(p); });
            writes(c, [&](const void* p) { wr.insert(p); });
        };
        add(i);
        size_t j = i + 1;
        for (; j < n && same_run(i, j); j++) {
            bool clash = false;
            reads(j, [&](const void* p) { clash = clash || wr.contains(p); });
            writes(j, [&](const void* p) { clash = clash || wr.contains(p) || rd.contains(p); });
            if (clash) break;
            add(j);
        }
        ends.push_back(j);
        i = j;
    }
    return ends;
}

// Last HIP error seen by this thread (for diagnostics through the C ABI).
const char* last_error_string();
void set_last_error(const std::string& s);

}  // namespace ecg
