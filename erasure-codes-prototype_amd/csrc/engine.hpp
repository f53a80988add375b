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
#include <atomic>
#include <memory>
#include <mutex>
#include <shared_mutex>
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

class Engine;

// A caller stream's identity for comparisons (program-set retirement, upload readiness).  hipStreamPerThread
// is ONE handle value that names a different stream on every thread, so it is keyed per thread: a serial
// number unique to the thread for the life of the process, shifted and tagged with bit 0 (real handles are
// aligned pointers, so no key equals one).  A set noted under such a key is covered only by its own thread --
// at a launch on hipStreamPerThread, or a cache miss on it -- where the handle names that very stream; a
// thread that exits leaves its sets to the graveyard (a cover on another thread's per-thread
// stream could fire while the noting thread's launch was still queued).
hipStream_t stream_key(hipStream_t st);

struct ProgramSet {
    Engine* owner = nullptr;  // its device memory (one block: tables + ids) goes back to owner's pool
    uint64_t serial = 0;      // unique per set (retirement names sets by it, not by address)
    void* mem = nullptr;
    size_t mem_class = 0;
    CoefTab* d_tabs = nullptr;
    int* d_src = nullptr;
    int* d_dst = nullptr;
    int nprog = 0, k = 0, m = 0, MT = 1, rtiles = 1;
    bool binary = false;
    // Retirement after eviction: the tables are freed only once every launch that reads them has completed.
    // A caller stream is never handed to the runtime after the call that passed it returns -- the caller
    // may destroy it, and the runtime crashes on a destroyed handle (hipEventRecord / hipStreamQuery
    // segfault, profiles/r04/stream/) -- and no event is recorded per launch either (a separate
    // hipEventRecord or a stop event bound to each launch cost ~3 us of host and GPU time per small launch,
    // profiles/r04/stream/).  Instead a launch only notes its stream handle (compared, never passed to
    // HIP).  Once the set is retired and nobody holds it, each noted stream gets a "cover" event recorded on
    // it the next time the library is handed that stream anyway (a later launch or cache miss on it: the
    // stream is alive then, and a record then follows every earlier launch on it).  The null stream is never
    // destroyed, so it is covered at once; hipStreamPerThread slots carry their thread's stream_key and are
    // covered from that thread only.  Slots hold stream_key()s.  A set whose streams are never
    // seen again (destroyed, or idle) waits in a bounded graveyard, emptied by a device synchronize when it
    // outgrows ECG_OPT_GRAVEYARD or on ecg_program_sets_reclaim.  Host-tier launches are not noted: those calls
    // wait for their own completion before they return.  More than kMaxStreams streams -> graveyard.
    static constexpr int kMaxStreams = 8;
    struct CoverEvent;
    struct StreamSlot {
        hipStream_t st;                     // compared, never passed to HIP
        std::shared_ptr<CoverEvent> cover;  // recorded on st after the set was retired
    };
    std::mutex smu;
    StreamSlot slots[kMaxStreams] = {};
    int nslots = 0;
    bool overflow = false;
    std::atomic<int> nslots_pub{0};  // slots[0, nslots_pub) have their stream set (lock-free launch check)
    void used_on(hipStream_t st) {  // launch path: note the caller stream (its stream_key)
        const int n = nslots_pub.load(std::memory_order_acquire);
        for (int i = 0; i < n; i++)
            if (slots[i].st == st) return;  // the common case: no lock
        std::lock_guard<std::mutex> lk(smu);
        for (int i = 0; i < nslots; i++)
            if (slots[i].st == st) return;
        if (nslots < kMaxStreams) {
            slots[nslots++].st = st;
            nslots_pub.store(nslots, std::memory_order_release);
        } else {
            overflow = true;
        }
    }
    // upload state (program_set): the tables are copied on the first requesting stream
    hipEvent_t ready_ev = nullptr;
    hipStream_t first_stream = nullptr;  // stream_key of the uploading stream, compared only
    std::atomic<bool> ready{false};
    void* pinned = nullptr;  // source of the asynchronous upload (pinned pool block, returned once ready)
    size_t pinned_class = 0;
    int ensure_ready(hipStream_t st);
    ~ProgramSet();  // returns the memory at once: only reached when no launch can still read the tables
};

class Engine {
public:
    static Engine& instance();  // engine of the calling thread's current HIP device

    int run_device(const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B,
                   hipStream_t stream);
    // The same with a shared (interned) plan: a call recorded in a batch scope keeps the pointer.
    int run_device(const std::shared_ptr<const std::vector<LinearOp>>& ops, uint8_t* const* blocks, int nblocks,
                   long long B, hipStream_t stream);
    int run_host(const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B);
    int run_strided(const std::vector<LinearOp>& progs, const int* d_prog_of_stripe, int S,
                    const void* in_base, long long in_sstride, long long in_bstride, void* out_base,
                    long long out_sstride, long long out_bstride, long long B, hipStream_t stream,
                    const int* d_stripe_of = nullptr);
    // apart: every call's outputs lie apart from its inputs (the grid-map hint, outputs_apart)
    int run_ptrs(const LinearOp& prog, const uint8_t* const* d_src, uint8_t* const* d_dst, int S, long long B,
                 bool aligned16, hipStream_t stream, bool apart = false);
    // One op over S calls' block pointers (host arrays): uploads the pointer tables, then run_ptrs.
    int run_ptr_batch(const LinearOp& op, const std::vector<const uint8_t* const*>& call_blocks, long long B,
                      hipStream_t stream);
    // Calls of one op shape with per-call ops (different coefficient matrices): ONE pointer-table launch
    // with a program per distinct matrix.
    int run_ptr_batch_multi(const std::vector<const LinearOp*>& ops, const std::vector<const uint8_t* const*>& calls,
                            long long B, hipStream_t stream);
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

    // The cached program set of `progs`, built (tables uploaded asynchronously on `st`) on a miss.  The
    // caller launches on `st` after ps->ensure_ready(st).
    std::shared_ptr<ProgramSet> program_set(const std::vector<LinearOp>& progs, int* status, hipStream_t st);
    std::shared_ptr<ProgramSet> program_set(const LinearOp* progs, size_t nprogs, int* status, hipStream_t st);
    int host_contexts() const;  // host-tier contexts created so far (pooled; bounded by concurrent calls)
    int device() const { return device_; }
    size_t cache_size();

    int launch_direct(const std::vector<LinearOp>& ops, uint8_t* const* blocks, long long B, hipStream_t stream);

    // Events (retirement covers, batch-scope ordering), pooled.  acquire_event creates on the current
    // device, which must be this engine's; release only an event no pending wait can still need recorded
    // again (a wait already enqueued refers to the record at the time of the wait).
    hipEvent_t acquire_event();
    void release_event(hipEvent_t ev);

    // After enqueueing a launch of `ps` on caller stream st (device and batched tiers): note the stream on
    // the set and, if retired sets wait for a cover on a stream hashing like st, cover them on st now.
    void note_launch(ProgramSet& ps, hipStream_t st) {
        const hipStream_t key = stream_key(st);
        ps.used_on(key);
        if (cover_mask_.load(std::memory_order_relaxed) & stream_bit(key)) cover_retired(st);
    }
    size_t retired_pending();  // evicted sets not yet freed (sweeps first; no synchronize)
    size_t reclaim();          // synchronize the device, free every retired set nobody holds; pending after

private:
    explicit Engine(int device);
    // latency: the blocks are host memory read over PCIe (zero-copy host tier) -> GF_MODE_INLINE_LAT
    // latency: the zero-copy host-tier variant; with flags (device view), it also posts completion flags
    // at flags[0, *n_flags) with value seq (GfLaunch::done_flags)
    // host_tier: `stream` is a leased host-tier stream and the call waits for the launch before it returns,
    // so the launch is not noted for retirement (ProgramSet::used_on)
    int launch_one(const LinearOp& op, uint8_t* const* blocks, long long B, hipStream_t stream, bool host_tier,
                   bool latency = false, unsigned* flags = nullptr, unsigned seq = 0, int* n_flags = nullptr);

    // Evicted sets wait here until nothing can read their tables: first until no caller holds them (no
    // further launch can be enqueued), then until the cover event of every stream they were launched on has
    // fired (ProgramSet: covers are recorded on a stream only while the library holds it from a caller).
    // Swept on every cache miss, with the miss's stream as `current`; no device-wide synchronize unless the
    // graveyard of sets that cannot be covered outgrows ECG_OPT_GRAVEYARD.
    void retire(std::vector<std::shared_ptr<ProgramSet>>&& evicted);
    void sweep_retired(hipStream_t current, bool has_current);
    void cover_retired(hipStream_t st);  // a launch on st (the caller's handle) hit the cover mask
    // under rmu_: true = the graveyard outgrew ECG_OPT_GRAVEYARD (the caller then runs sync_and_free_unheld)
    bool sweep_locked(hipStream_t current, bool has_current, std::vector<std::shared_ptr<ProgramSet>>& dead);
    size_t sync_and_free_unheld();
    // Stream handles are 16-byte aligned pointers (their low 4 bits carry nothing); hipStreamPerThread keys
    // (stream_key: serial << 1 | 1) are small odd numbers whose information sits in the low bits, so they
    // are hashed whole -- shifted like handles, threads 1-7 all landed on the null stream's bit.
    static uint64_t stream_bit(hipStream_t st) {
        const uintptr_t v = (uintptr_t)st;
        return 1ull << ((((v & 1) ? v : v >> 4) * 0x9E3779B97F4A7C15ull) >> 58);
    }
    // Device memory of program tables comes from a pool of power-of-two blocks, so a steady stream of new
    // programs (a proxy's open set of repair matrices) neither allocates nor frees device memory --
    // hipFree synchronizes the device.  Uploads go through a private non-blocking stream.
    void* acquire_tables(size_t bytes, size_t* cls, hipError_t* err);
    void release_tables(void* p, size_t cls);
    // the same for the pinned host blocks the uploads are copied from (a pageable source would make
    // the asynchronous copy wait for the stream's earlier work)
    void* acquire_pinned(size_t bytes, size_t* cls, hipError_t* err);
    void release_pinned(void* p, size_t cls);
    friend struct ProgramSet;

    int device_;
    struct CacheEntry {
        std::shared_ptr<ProgramSet> ps;
        std::unique_ptr<std::atomic<uint64_t>> last_use;  // updated under the shared lock
    };
    // hits (every launch) take the lock shared; builds and evictions take it exclusively
    std::shared_mutex mu_;
    std::atomic<uint64_t> tick_{0};
    std::unordered_map<std::string, CacheEntry> cache_;  // LRU-bounded by ECG_OPT_PROGRAM_CACHE
    std::mutex rmu_;
    std::vector<std::shared_ptr<ProgramSet>> retired_;
    // unheld retired sets waiting for a cover on each stream key (rebuilt by every sweep; weak: the sets are
    // owned by retired_), and the stream_bit of every key in it
    std::unordered_map<hipStream_t, std::vector<std::weak_ptr<ProgramSet>>> waiting_;
    std::atomic<uint64_t> cover_mask_{0};
    std::mutex pmu_;
    std::unordered_map<size_t, std::vector<void*>> pool_, pinned_pool_;
    std::vector<hipEvent_t> event_pool_;
    size_t pooled_bytes_ = 0, pinned_pooled_bytes_ = 0;
};

// Deferred-batch scope of the calling thread (ecg_batch_begin / ecg_batch_end).  Inside a scope,
// device-tier calls (run_device: ecg_dev_matrix_*, ErasureCode objects on HBM buffers) are recorded
// instead of launched.  batch_flush() then
//   1. composes away scratch blocks (batch_scratch): a block written and later read inside the scope
//      whose memory the caller declared scratch is never written -- its readers take the linear map
//      that produced it instead (the helper partial + main partial + perform_addition sequence of a
//      partial-decoding repair becomes one region product per repair, compose_scratch below);
//   2. groups the calls (schedule_groups below): calls with the same plan, block size, stream and
//      device join one group unless a data dependence orders them apart, and each group goes out as
//      ONE launch per op -- strided when its blocks form one strided batch, a pointer-table launch
//      otherwise.  Groups launch in an order that respects every read/write dependence of the recorded
//      sequence, so the result is the sequential result.
// Host-tier and batched calls flush first, so call order is kept.  A flush launches each group on its
// engine's device (the calling thread's device is restored after).  If a launch fails, the flush stops
// there and returns the error; the calls of that group and of every later group are dropped (not
// retried by a later flush).
int batch_begin();
int batch_flush();
int batch_end();
bool batch_active();
// Host-tier calls of the scope are recorded too (ecg_batch_defer_host): see DeferScope::hq in engine.cpp.
int batch_defer_host(int on);
int record_host(Engine* eng, const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B);
int host_flush();
int batch_flush_all();  // both queues (ecg_batch_flush)
// Declare [p, p + bytes) scratch for the rest of the current scope (ECG_EINVAL outside a scope).
int batch_scratch(const void* p, size_t bytes);
// Flush this thread's recorded calls, if any (entry points that launch directly call it first, so a
// recorded call never runs after a later direct launch).
int batch_flush_pending();
// What the last flush of this thread did: calls recorded, calls after scratch composition, launches
// (groups x ops; byte-path tails not counted), scratch expressions materialised (written for real).
struct FlushStats {
    long long recorded = 0, composed = 0, groups = 0, launches = 0, materialised = 0;
};
FlushStats last_flush_stats();

// One recorded device-tier call: its plan (shared by calls with an equal plan) over its block space.
struct DeferredCall {
    Engine* eng;
    hipStream_t st;
    long long B;
    std::shared_ptr<const std::vector<LinearOp>> ops;
    std::vector<uint8_t*> blocks;  // device pointers
};

// Scratch ranges of a scope (merged, disjoint).  A block [p, p + B) is scratch if one range holds it.
class ScratchRanges {
public:
    void add(uintptr_t lo, uintptr_t hi);
    bool holds(const void* p, long long B) const;
    bool empty() const { return r_.empty(); }
    void clear() { r_.clear(); }

private:
    std::vector<std::pair<uintptr_t, uintptr_t>> r_;  // sorted by start, disjoint, [lo, hi)
};

// Scratch composition (pure host logic, no HIP; fuzzed in tests/sanitize/host_fuzz.cpp against a
// sequential interpreter).  Walks the recorded calls in order, keeping for every scratch block written
// so far the linear combination of real blocks it holds (an "expression").  A call reading a scratch
// block with an expression reads that combination's blocks instead (coefficients multiplied out over
// GF(2^8)); a call writing a scratch block only records the expression.  An expression is written for
// real ("materialised") before any block it reads is overwritten, when a reader runs on another
// stream / device / block size, and -- unless `scope_end` -- for every expression left at the end
// (a mid-scope flush must leave memory as the sequential calls would).  At scope end unconsumed
// scratch contents are undefined: that is the contract of batch_scratch.  Blocks are compared by
// address, as in the hazard check (blocks of one scope are identical or disjoint).  Calls that touch
// neither scratch nor an expression pass through unchanged (their plan pointer kept).
std::vector<DeferredCall> compose_scratch(std::vector<DeferredCall>&& q, const ScratchRanges& scratch,
                                          bool scope_end, long long* materialised);

// Block addresses are often aligned to the block size (1 MiB and up): a full 64-bit mix (splitmix64's
// finaliser) so that their low bits, which pick the slot, are not mostly zero.
inline size_t ptr_hash(uintptr_t p) {
    unsigned long long x = (unsigned long long)p;
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (size_t)x;
}

// Open-addressing map block address -> the latest group (index + 1) that read / wrote it, for the
// flush's scheduler.  0 = never touched.
class PtrGroups {
public:
    struct Slot {
        uintptr_t p;
        int rd, wr;
    };
    Slot& at(const void* ptr) {
        if ((count_ + 1) * 2 > slots_.size()) grow();
        const uintptr_t p = (uintptr_t)ptr;
        for (size_t i = hash(p) & mask_;; i = (i + 1) & mask_) {
            if (slots_[i].p == p) return slots_[i];
            if (slots_[i].p == 0) {
                slots_[i] = Slot{p, 0, 0};
                count_++;
                return slots_[i];
            }
        }
    }
    // empty, with room for n addresses without growing (the flush's scheduler reuses one per thread)
    void reset(size_t n) {
        size_t want = 1024;
        while (want < 4 * n) want <<= 1;
        if (slots_.size() < want) {
            slots_.assign(want, Slot{0, 0, 0});
            mask_ = want - 1;
        } else if (count_) {
            std::fill(slots_.begin(), slots_.end(), Slot{0, 0, 0});
        }
        count_ = 0;
    }
    int last_write(const void* ptr) const { const Slot* s = find(ptr); return s ? s->wr : 0; }
    const Slot* find_slot(const void* ptr) const { return find(ptr); }
    int last_touch(const void* ptr) const { const Slot* s = find(ptr); return s ? std::max(s->rd, s->wr) : 0; }

private:
    const Slot* find(const void* ptr) const {
        if (slots_.empty()) return nullptr;
        const uintptr_t p = (uintptr_t)ptr;
        for (size_t i = hash(p) & mask_;; i = (i + 1) & mask_) {
            if (slots_[i].p == p) return &slots_[i];
            if (slots_[i].p == 0) return nullptr;
        }
    }
    static size_t hash(uintptr_t p) { return ptr_hash(p); }
    void grow() {
        std::vector<Slot> old;
        old.swap(slots_);
        slots_.assign(old.empty() ? 1024 : old.size() * 2, Slot{0, 0, 0});
        mask_ = slots_.size() - 1;
        count_ = 0;
        for (const Slot& s : old)
            if (s.p) at((const void*)s.p) = s;
    }
    std::vector<Slot> slots_;
    size_t mask_ = 0, count_ = 0;
};

// Grouping of the flush (pure host logic, no HIP; fuzzed against a quadratic legality check in
// tests/sanitize/host_fuzz.cpp).  Calls [0, n) in program order; key(c) >= 0 names the call's plan
// class (same plan or single-op shape, block size, stream, device).  Each call joins the EARLIEST group of
// its key that comes after every group holding an earlier call it depends on (one that writes a block it
// reads or writes, or reads a block it writes); if there is none it opens a new group at the end.
// Launching the groups in index order, each group's calls in one launch, therefore respects every
// dependence of the program order (two dependent calls always sit in groups i < j), and independent calls
// of one plan -- the reference's per-stripe loop, even with several plans interleaved per stripe -- share a
// launch.  Earliest, not latest: in a two-block repair whose second plan reads the block its first plan
// rebuilt (handle_repair.cpp per plan), every stripe's first plan shares one group and every second plan
// the next, instead of a new pair of groups per stripe (a launch per stripe).  A call placed before a later
// group of its key depends on nothing in between, and calls after it see its group in `seen`.
// reads(c, f) / writes(c, f) call f(address) per block call c reads / writes.  Returns the groups,
// each listing its calls in program order.
template <class Key, class Reads, class Writes>
std::vector<std::vector<size_t>> schedule_groups(size_t n, Key key, Reads reads, Writes writes) {
    std::vector<std::vector<size_t>> groups;
    std::vector<std::vector<int>> of_key;  // key -> its groups' index + 1, ascending
    thread_local PtrGroups seen;
    seen.reset(4 * n);
    for (size_t c = 0; c < n; c++) {
        int lo = 0;  // the call must go into a group with index + 1 > lo
        reads(c, [&](const void* p) { lo = std::max(lo, seen.last_write(p)); });
        writes(c, [&](const void* p) { lo = std::max(lo, seen.last_touch(p)); });
        const int kc = key(c);
        if ((size_t)kc >= of_key.size()) of_key.resize((size_t)kc + 1);
        std::vector<int>& mine = of_key[(size_t)kc];
        const auto it = std::upper_bound(mine.begin(), mine.end(), lo);
        int g1;
        if (it != mine.end()) {
            g1 = *it;
        } else {
            groups.emplace_back();
            g1 = (int)groups.size();
            mine.push_back(g1);
        }
        groups[(size_t)g1 - 1].push_back(c);
        reads(c, [&](const void* p) { PtrGroups::Slot& s = seen.at(p); s.rd = std::max(s.rd, g1); });
        writes(c, [&](const void* p) { PtrGroups::Slot& s = seen.at(p); s.wr = std::max(s.wr, g1); });
    }
    return groups;
}

// Resident call worker of the calling thread's device (ECG_OPT_CALL_WORKER): calls, launches, relaunches,
// off now (set-up failure, or a cooldown after a timed-out call).
int call_worker_stats(long long* calls, long long* launches, long long* relaunches, int* disabled);

// Last HIP error seen by this thread (for diagnostics through the C ABI).
const char* last_error_string();
void set_last_error(const std::string& s);

}  // namespace ecg
