// GF(2^8) region engine.  See engine.hpp.
#include "engine.hpp"

#include <emmintrin.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <numeric>
#include <thread>
#include <tuple>

#include "gf256.hpp"

namespace ecg {

namespace {

thread_local std::string t_last_error;

#define ECG_HIP(call)                                                                        \
    do {                                                                                     \
        hipError_t _e = (call);                                                              \
        if (_e != hipSuccess) {                                                              \
            set_last_error(std::string(#call) + ": " + hipGetErrorString(_e));               \
            return ECG_EHIP;                                                                 \
        }                                                                                    \
    } while (0)

constexpr int kMaxDevices = 64;
std::mutex g_engines_mu;
std::atomic<Engine*> g_engines[kMaxDevices] = {};

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// One call's outputs lie apart from its inputs: none inside the span of its input blocks or the m blocks
// just past it (where an encode into [k+m][B] stripes or an in-place decode writes).  The pointer-table
// launch's grid-map hint (gf_kernels.hip outputs_in_stripe): speed only, never correctness.
static bool outputs_apart(const uint8_t* const* src, int k, const uint8_t* const* dst, int m, long long B) {
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    for (int j = 0; j < k; j++) {
        lo = std::min(lo, (uintptr_t)src[j]);
        hi = std::max(hi, (uintptr_t)src[j] + (uintptr_t)B);
    }
    for (int q = 0; q < m; q++) {
        const uintptr_t d = (uintptr_t)dst[q];
        if (d + (uintptr_t)B > lo && d < hi + (uintptr_t)m * (uintptr_t)B) return false;
    }
    return true;
}

// Host-tier state: a non-blocking stream, a growable device scratch, a pinned staging area and the
// host-batch pipeline's streams and slots.  Contexts are pooled per device and LEASED for the duration
// of one synchronous host-tier call, so these resources are bounded by the number of calls in flight
// at once -- not by the number of threads that ever called.  (The reference's proxy runs every SET on
// a new detached thread, proxy.cpp:416-419; per-thread state would leak a stream, scratch and pinned
// memory per request.)  Contexts live for the process.
struct HostCtx {
    hipStream_t stream = nullptr;
    uint8_t* scratch = nullptr;
    size_t cap = 0;
    // host-batch pipeline: 3 streams, 3 device slots
    hipStream_t pstream[3] = {nullptr, nullptr, nullptr};
    hipEvent_t in_done[3] = {}, comp_done[3] = {}, out_done[3] = {};
    bool pipe_ready = false;
    uint8_t* pslot = nullptr;
    size_t pslot_cap = 0;
    // small host calls: one pinned staging area mirroring the device scratch
    uint8_t* pinned = nullptr;      // host view
    uint8_t* pinned_dev = nullptr;  // device view (mapped, fine-grained)
    size_t pinned_cap = 0;
    // zero-copy calls: completion flags the kernels post and the host polls (mapped, fine-grained)
    unsigned* flags = nullptr;
    unsigned* flags_dev = nullptr;
    unsigned seq = 0;
    unsigned unreaped = 0;  // flagged calls since the stream was last queried
};
constexpr int kFlagSlots = 4096;

std::mutex g_ctx_mu[kMaxDevices];
// never destroyed (process lifetime, like the engines): no teardown-order hazard with late callers
std::vector<HostCtx*>* const g_ctx_free = new std::vector<HostCtx*>[kMaxDevices];
int g_ctx_created[kMaxDevices] = {};

class CtxLease {
public:
    explicit CtxLease(int device) : dev_(device) {
        std::lock_guard<std::mutex> lk(g_ctx_mu[dev_]);
        if (!g_ctx_free[dev_].empty()) {
            c_ = g_ctx_free[dev_].back();
            g_ctx_free[dev_].pop_back();
        } else {
            c_ = new HostCtx();
            g_ctx_created[dev_]++;
        }
    }
    ~CtxLease() {
        if (!idle_) {
            // a call that failed part-way may have left copies in flight: drain before the next lessee
            if (c_->stream) (void)hipStreamSynchronize(c_->stream);
            for (hipStream_t s : c_->pstream)
                if (s) (void)hipStreamSynchronize(s);
        }
        std::lock_guard<std::mutex> lk(g_ctx_mu[dev_]);
        g_ctx_free[dev_].push_back(c_);
    }
    CtxLease(const CtxLease&) = delete;
    CtxLease& operator=(const CtxLease&) = delete;
    HostCtx& operator*() { return *c_; }
    int done() {  // the call completed and synchronised its streams
        idle_ = true;
        return ECG_OK;
    }

private:
    int dev_;
    HostCtx* c_;
    bool idle_ = false;
};

}  // namespace

const char* last_error_string() { return t_last_error.c_str(); }
void set_last_error(const std::string& s) { t_last_error = s; }

// Freed without waiting: a set that was ever launched is destroyed only by sweep_retired(), after its
// launches completed; any other (a lost insertion race, a failed build) was never launched.
ProgramSet::~ProgramSet() {
    if (ready_ev) {
        // a set dropped before its upload was seen complete (a lost insertion race): the copy must land
        // before the memory is reused
        if (!ready.load(std::memory_order_acquire)) (void)hipEventSynchronize(ready_ev);
        (void)hipEventDestroy(ready_ev);
    }
    if (pinned) owner->release_pinned(pinned, pinned_class);
    if (mem) owner->release_tables(mem, mem_class);
}

// A retirement cover: an event recorded on one stream after the set was retired; back to the pool when the
// last set it covers is freed (it has fired by then, or the device was synchronized).
struct ProgramSet::CoverEvent {
    Engine* eng;
    hipEvent_t ev;
    ~CoverEvent() { eng->release_event(ev); }
};

hipEvent_t Engine::acquire_event() {
    {
        std::lock_guard<std::mutex> lk(pmu_);
        if (!event_pool_.empty()) {
            hipEvent_t ev = event_pool_.back();
            event_pool_.pop_back();
            return ev;
        }
    }
    hipEvent_t ev = nullptr;
    return hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess ? ev : nullptr;
}

void Engine::release_event(hipEvent_t ev) {
    std::lock_guard<std::mutex> lk(pmu_);
    event_pool_.push_back(ev);
}

// Before a launch on `st` reads the set's tables: once the upload event has fired the set is ready for
// every stream; until then a launch on another stream than the uploading one waits for the event.
int ProgramSet::ensure_ready(hipStream_t st) {
    if (ready.load(std::memory_order_acquire)) return ECG_OK;
    const hipError_t q = hipEventQuery(ready_ev);
    if (q == hipSuccess) {
        std::lock_guard<std::mutex> lk(smu);  // one thread hands the pinned source back
        if (!ready.load(std::memory_order_relaxed)) {
            if (pinned) owner->release_pinned(pinned, pinned_class);
            pinned = nullptr;
            ready.store(true, std::memory_order_release);
        }
        return ECG_OK;
    }
    if (q != hipErrorNotReady) return ECG_EHIP;
    if (stream_key(st) != first_stream && hipStreamWaitEvent(st, ready_ev, 0) != hipSuccess) return ECG_EHIP;
    return ECG_OK;
}

void* Engine::acquire_tables(size_t bytes, size_t* cls, hipError_t* err) {
    size_t c = 256;
    while (c < bytes) c <<= 1;
    *cls = c;
    *err = hipSuccess;
    {
        std::lock_guard<std::mutex> lk(pmu_);
        auto it = pool_.find(c);
        if (it != pool_.end() && !it->second.empty()) {
            void* p = it->second.back();
            it->second.pop_back();
            pooled_bytes_ -= c;
            return p;
        }
    }
    void* p = nullptr;
    *err = hipMalloc(&p, c);
    return *err == hipSuccess ? p : nullptr;
}

void* Engine::acquire_pinned(size_t bytes, size_t* cls, hipError_t* err) {
    size_t c = 256;
    while (c < bytes) c <<= 1;
    *cls = c;
    *err = hipSuccess;
    {
        std::lock_guard<std::mutex> lk(pmu_);
        auto it = pinned_pool_.find(c);
        if (it != pinned_pool_.end() && !it->second.empty()) {
            void* p = it->second.back();
            it->second.pop_back();
            pinned_pooled_bytes_ -= c;
            return p;
        }
    }
    void* p = nullptr;
    *err = hipHostMalloc(&p, c, hipHostMallocDefault);
    return *err == hipSuccess ? p : nullptr;
}

void Engine::release_pinned(void* p, size_t cls) {
    constexpr size_t kPinnedCap = 16 << 20;
    {
        std::lock_guard<std::mutex> lk(pmu_);
        if (pinned_pooled_bytes_ + cls <= kPinnedCap) {
            pinned_pool_[cls].push_back(p);
            pinned_pooled_bytes_ += cls;
            return;
        }
    }
    (void)hipHostFree(p);
}

void Engine::release_tables(void* p, size_t cls) {
    constexpr size_t kPoolCap = 64 << 20;  // beyond this, blocks are freed (rare: a cache of large programs)
    {
        std::lock_guard<std::mutex> lk(pmu_);
        if (pooled_bytes_ + cls <= kPoolCap) {
            pool_[cls].push_back(p);
            pooled_bytes_ += cls;
            return;
        }
    }
    (void)hipFree(p);
}

void Engine::retire(std::vector<std::shared_ptr<ProgramSet>>&& evicted) {
#ifndef ECG_TEST_TSAN_SEEDED_RACE  // test hook: tools/tsan_host.sh seeded must report this unlocked push as a race
    std::lock_guard<std::mutex> lk(rmu_);
#endif
    for (auto& ps : evicted) retired_.push_back(std::move(ps));
}

hipStream_t stream_key(hipStream_t st) {
#ifdef ECG_TEST_PER_THREAD_SHARED_KEY  // test hook: round 4's one key for every thread's per-thread stream
    return st;                         // (tools/tsan_host.sh sharedkey must report a device-time hazard)
#endif
    if (st != hipStreamPerThread) return st;
    static std::atomic<uintptr_t> next{1};
    static thread_local const uintptr_t key = (next.fetch_add(1, std::memory_order_relaxed) << 1) | 1;
    return (hipStream_t)key;
}

// One pass over the retired sets (ProgramSet's retirement comment):
//   1. every unheld set's uncovered stream that may be named now -- `current` (a stream the caller handed
//      the library in the call in progress) or a stream that is never destroyed -- gets a cover event,
//      one record per stream per pass;
//   2. sets whose covers (and upload) have all fired are freed;
//   3. the cover mask is rebuilt from the streams still waiting;
//   4. unheld sets that cannot be covered (streams not seen again, overflow) beyond ECG_OPT_GRAVEYARD: the
//      caller synchronizes the device outside the lock and frees them (sync_and_free_unheld).
void Engine::sweep_retired(hipStream_t current, bool has_current) {
    bool over = false;
    {
        std::vector<std::shared_ptr<ProgramSet>> dead;  // destroyed after the lock is released
        std::lock_guard<std::mutex> lk(rmu_);
        over = sweep_locked(current, has_current, dead);
    }
    if (over) (void)sync_and_free_unheld();  // the graveyard outgrew ECG_OPT_GRAVEYARD
}

// A launch on st hit the cover mask: cover the unheld retired sets that wait for st's key (one event record
// on st, the caller's handle: for hipStreamPerThread, this thread's stream, the one the key names).
void Engine::cover_retired(hipStream_t st) {
    const hipStream_t key = stream_key(st);
    std::lock_guard<std::mutex> lk(rmu_);
    auto it = waiting_.find(key);
    if (it == waiting_.end()) return;  // another stream with the same mask bit
    std::shared_ptr<ProgramSet::CoverEvent> cover;
    auto& v = it->second;
    for (size_t i = 0; i < v.size();) {
        std::shared_ptr<ProgramSet> ps = v[i].lock();
        if (ps && ps.use_count() > 2) {  // still held by a caller (beyond retired_ and `ps`)
            i++;
            continue;
        }
        if (ps) {
            if (!cover) {
                hipEvent_t ev = acquire_event();
                if (!ev) return;
                if (hipEventRecord(ev, st) != hipSuccess) {
                    release_event(ev);
                    return;
                }
                cover = std::make_shared<ProgramSet::CoverEvent>(ProgramSet::CoverEvent{this, ev});
            }
            std::lock_guard<std::mutex> sk(ps->smu);
            for (int e = 0; e < ps->nslots; e++)
                if (ps->slots[e].st == key && !ps->slots[e].cover) ps->slots[e].cover = cover;
        }
        v[i] = std::move(v.back());
        v.pop_back();
    }
    if (v.empty()) {
        waiting_.erase(it);
        uint64_t mask = 0;
        for (auto& kv : waiting_) mask |= stream_bit(kv.first);
        cover_mask_.store(mask, std::memory_order_relaxed);
    }
}

bool Engine::sweep_locked(hipStream_t current, bool has_current, std::vector<std::shared_ptr<ProgramSet>>& dead) {
    if (retired_.empty()) {
        waiting_.clear();
        cover_mask_.store(0, std::memory_order_relaxed);
        return false;
    }
    // slots hold stream keys: a slot is covered on `current` (the caller's handle, which names the slot's
    // stream in this thread) when its key is current's, and at once when it is the null stream
    const hipStream_t cur_key = has_current ? stream_key(current) : nullptr;
    std::shared_ptr<ProgramSet::CoverEvent> made[2];  // current, null stream
    auto cover_for = [&](hipStream_t key) -> std::shared_ptr<ProgramSet::CoverEvent> {
        const int i = (has_current && key == cur_key) ? 0 : key == nullptr ? 1 : -1;
        if (i < 0) return nullptr;
        if (!made[i]) {
            hipEvent_t ev = acquire_event();
            if (!ev) return nullptr;
            if (hipEventRecord(ev, i == 0 ? current : nullptr) != hipSuccess) {
                release_event(ev);
                return nullptr;
            }
            made[i] = std::make_shared<ProgramSet::CoverEvent>(ProgramSet::CoverEvent{this, ev});
        }
        return made[i];
    };
    size_t graveyard = 0;
    waiting_.clear();
    for (size_t i = 0; i < retired_.size();) {
        ProgramSet& ps = *retired_[i];
        const bool unheld = retired_[i].use_count() == 1;
        bool done = unheld;
        {
            std::lock_guard<std::mutex> sk(ps.smu);
            for (int e = 0; e < ps.nslots; e++) {
                ProgramSet::StreamSlot& sl = ps.slots[e];
                if (!sl.cover && unheld && (sl.st == nullptr || (has_current && sl.st == cur_key)))
                    sl.cover = cover_for(sl.st);
                if (!sl.cover) {
                    if (unheld) waiting_[sl.st].push_back(retired_[i]);
                    done = false;
                } else if (done) {
                    done = hipEventQuery(sl.cover->ev) == hipSuccess;
                }
            }
            if (ps.overflow) done = false;
            if (done && !ps.ready.load(std::memory_order_acquire)) done = hipEventQuery(ps.ready_ev) == hipSuccess;
        }
        if (done) {
            dead.push_back(std::move(retired_[i]));
            retired_[i] = std::move(retired_.back());
            retired_.pop_back();
            continue;
        }
        if (unheld) graveyard++;
        i++;
    }
    uint64_t mask = 0;
    for (auto& kv : waiting_) mask |= stream_bit(kv.first);
    cover_mask_.store(mask, std::memory_order_relaxed);
    return graveyard > (size_t)get_option(ECG_OPT_GRAVEYARD);
}

// Synchronize the engine's device WITHOUT holding the retirement lock (launches that hit the cover mask
// take it), then free the sets that nobody held before the synchronize began: their launches were all
// enqueued by then.  Sets are named by serial number, not address (a freed set's address may be reused).
size_t Engine::sync_and_free_unheld() {
    std::vector<uint64_t> before;
    {
        std::lock_guard<std::mutex> lk(rmu_);
        for (auto& ps : retired_)
            if (ps.use_count() == 1) before.push_back(ps->serial);
    }
    int caller_dev = -1;
    (void)hipGetDevice(&caller_dev);
    const bool switched = caller_dev != device_ && hipSetDevice(device_) == hipSuccess;
    const bool synced = hipDeviceSynchronize() == hipSuccess;
    if (switched) (void)hipSetDevice(caller_dev);
    std::vector<std::shared_ptr<ProgramSet>> dead;
    std::lock_guard<std::mutex> lk(rmu_);
    if (synced) {
        std::sort(before.begin(), before.end());
        for (size_t i = 0; i < retired_.size();) {
            if (std::binary_search(before.begin(), before.end(), retired_[i]->serial)) {
                dead.push_back(std::move(retired_[i]));
                retired_[i] = std::move(retired_.back());
                retired_.pop_back();
                continue;
            }
            i++;
        }
    }
    (void)sweep_locked(nullptr, false, dead);  // rebuilds the waiting index and the cover mask
    return retired_.size();
}

size_t Engine::retired_pending() {
    std::vector<std::shared_ptr<ProgramSet>> dead;
    std::lock_guard<std::mutex> lk(rmu_);
    (void)sweep_locked(nullptr, false, dead);
    return retired_.size();
}

size_t Engine::reclaim() { return sync_and_free_unheld(); }

Engine::Engine(int device) : device_(device) {}

Engine& Engine::instance() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDevices) dev = 0;
    if (Engine* e = g_engines[dev].load(std::memory_order_acquire)) return *e;  // every call: no lock
    std::lock_guard<std::mutex> lk(g_engines_mu);
    if (!g_engines[dev].load(std::memory_order_relaxed))
        g_engines[dev].store(new Engine(dev), std::memory_order_release);  // lives for the process
    return *g_engines[dev].load(std::memory_order_relaxed);
}

int Engine::host_contexts() const {
    std::lock_guard<std::mutex> lk(g_ctx_mu[device_]);
    return g_ctx_created[device_];
}

size_t Engine::cache_size() {
    std::shared_lock<std::shared_mutex> lk(mu_);
    return cache_.size();
}

std::shared_ptr<ProgramSet> Engine::program_set(const std::vector<LinearOp>& progs, int* status, hipStream_t st) {
    return program_set(progs.data(), progs.size(), status, st);
}

std::shared_ptr<ProgramSet> Engine::program_set(const LinearOp* progs, size_t nprogs, int* status, hipStream_t st) {
    *status = ECG_OK;
    if (nprogs == 0) {
        *status = ECG_EINVAL;
        return nullptr;
    }
    const int k = progs[0].k_in(), m = progs[0].m_out();
    if (k < 1 || m < 1) {
        *status = ECG_EINVAL;
        return nullptr;
    }
    thread_local std::string key;  // per thread: no allocation per lookup
    key.clear();
    key.reserve(16 + nprogs * (size_t)(k * m + 4 * (k + m)));
    auto put = [&](const void* p, size_t n) { key.append((const char*)p, n); };
    const int np = (int)nprogs;
    put(&k, 4);
    put(&m, 4);
    put(&np, 4);
    bool binary = true;
    for (size_t pi = 0; pi < nprogs; pi++) {
        const LinearOp& op = progs[pi];
        if (op.k_in() != k || op.m_out() != m || op.coef.size() != (size_t)k * m) {
            *status = ECG_EINVAL;
            return nullptr;
        }
        put(op.coef.data(), op.coef.size());
        put(op.src_ids.data(), op.src_ids.size() * 4);
        put(op.dst_ids.data(), op.dst_ids.size() * 4);
        binary &= op_is_binary(op);
    }
    {
        std::shared_lock<std::shared_mutex> lk(mu_);
        auto it = cache_.find(key);
        if (it != cache_.end()) {
            it->second.last_use->store(tick_.fetch_add(1, std::memory_order_relaxed) + 1, std::memory_order_relaxed);
            return it->second.ps;
        }
    }
    auto ps = std::make_shared<ProgramSet>();
    static std::atomic<uint64_t> serials{0};
    ps->serial = ++serials;
    ps->nprog = np;
    ps->k = k;
    ps->m = m;
    ps->MT = std::min(m, binary ? kMaxMTBin : kMaxMT);
    ps->rtiles = (m + ps->MT - 1) / ps->MT;
    ps->binary = binary;
    const size_t per_prog = (size_t)ps->rtiles * k * ps->MT;
    std::vector<CoefTab> tabs(per_prog * np);
    std::vector<int> src((size_t)np * k), dst((size_t)np * m);
    for (int pi = 0; pi < np; pi++) {
        const LinearOp& op = progs[pi];
        for (int rt = 0; rt < ps->rtiles; rt++)
            for (int j = 0; j < k; j++)
                for (int p = 0; p < ps->MT; p++) {
                    const int row = rt * ps->MT + p;
                    const int c = row < m ? op.coef[(size_t)row * k + j] : 0;
                    make_coef_tab(c, &tabs[pi * per_prog + ((size_t)rt * k + j) * ps->MT + p]);
                }
        std::copy(op.src_ids.begin(), op.src_ids.end(), src.begin() + (size_t)pi * k);
        std::copy(op.dst_ids.begin(), op.dst_ids.end(), dst.begin() + (size_t)pi * m);
    }
    auto fail = [&](hipError_t e, const char* what) {
        set_last_error(std::string(what) + ": " + hipGetErrorString(e));
        *status = ECG_EHIP;
        return nullptr;
    };
    hipError_t e;
    // one device block: tables, then source ids, then destination ids
    const size_t tab_bytes = tabs.size() * sizeof(CoefTab), src_off = tab_bytes,
                 dst_off = src_off + ((src.size() * sizeof(int) + 15) & ~(size_t)15),
                 total = dst_off + dst.size() * sizeof(int);
    std::vector<uint8_t> host(total, 0);
    memcpy(host.data(), tabs.data(), tab_bytes);
    memcpy(host.data() + src_off, src.data(), src.size() * sizeof(int));
    memcpy(host.data() + dst_off, dst.data(), dst.size() * sizeof(int));
    ps->owner = this;
    ps->mem = acquire_tables(total, &ps->mem_class, &e);
    if (!ps->mem) return fail(e, "hipMalloc(program tables)");
    ps->d_tabs = (CoefTab*)ps->mem;
    ps->d_src = (int*)((uint8_t*)ps->mem + src_off);
    ps->d_dst = (int*)((uint8_t*)ps->mem + dst_off);
    // The upload goes on the requesting stream, asynchronously, ahead of the launch that needs it: no
    // host wait, and no other stream involved (streams share the runtime's few hardware queues, so a
    // private upload stream could sit behind another thread's queued work).  Launches on other streams
    // wait for `ready_ev` until it has fired (ensure_ready).  The host bytes stay with the set until then.
    if ((e = hipEventCreateWithFlags(&ps->ready_ev, hipEventDisableTiming)) != hipSuccess)
        return fail(e, "hipEventCreate(program tables)");
    ps->pinned = acquire_pinned(total, &ps->pinned_class, &e);
    if (!ps->pinned) return fail(e, "hipHostMalloc(program tables)");
    memcpy(ps->pinned, host.data(), total);
    ps->first_stream = stream_key(st);
    if ((e = hipMemcpyAsync(ps->mem, ps->pinned, total, hipMemcpyHostToDevice, st)) != hipSuccess) {
        (void)hipStreamSynchronize(st);
        return fail(e, "hipMemcpyAsync(program tables)");
    }
    if ((e = hipEventRecord(ps->ready_ev, st)) != hipSuccess) {
        (void)hipStreamSynchronize(st);  // the copy may be in flight: the memory must not go back yet
        ps->ready.store(true);
        return fail(e, "hipEventRecord(program tables)");
    }
    std::vector<std::shared_ptr<ProgramSet>> evicted;  // retired outside the lock
    {
        std::unique_lock<std::shared_mutex> lk(mu_);
        auto it = cache_.find(key);
        if (it != cache_.end()) {  // another thread won the race
            it->second.last_use->store(++tick_, std::memory_order_relaxed);
            return it->second.ps;
        }
        const size_t cap = (size_t)std::max(2LL, get_option(ECG_OPT_PROGRAM_CACHE));
        if (cache_.size() >= cap) {  // keep the cap / 2 most recently used programs
            std::vector<uint64_t> uses;
            uses.reserve(cache_.size());
            for (auto& kv : cache_) uses.push_back(kv.second.last_use->load(std::memory_order_relaxed));
            const size_t drop = cache_.size() - cap / 2;
            std::nth_element(uses.begin(), uses.begin() + drop, uses.end());
            const uint64_t cut = uses[drop];
            for (auto i = cache_.begin(); i != cache_.end();) {
                if (i->second.last_use->load(std::memory_order_relaxed) < cut) {
                    evicted.push_back(std::move(i->second.ps));
                    i = cache_.erase(i);
                } else {
                    ++i;
                }
            }
        }
        cache_.emplace(key, CacheEntry{ps, std::make_unique<std::atomic<uint64_t>>(++tick_)});
    }
    if (!evicted.empty()) retire(std::move(evicted));
    sweep_retired(st, true);  // st: the caller's stream, alive for this call
    return ps;
}

// One op over block pointers (device addresses), any k_in / m_out.  Ops that fit the kernel arguments
// carry their pointers inline; wider ones (k_in > 128 or m_out > 32) go through an uploaded pointer
// table (run_ptr_batch with one call), still asynchronous.
int Engine::launch_one(const LinearOp& op, uint8_t* const* blocks, long long B, hipStream_t st, bool host_tier,
                       bool latency, unsigned* flags, unsigned seq, int* n_flags) {
    if (n_flags) *n_flags = 0;
    if (op.m_out() == 0 || B == 0) return ECG_OK;
    if (op.k_in() == 0) {  // composed row of zeros: the library writes zero bytes
        for (int d : op.dst_ids) ECG_HIP(hipMemsetAsync(blocks[d], 0, (size_t)B, st));
        return ECG_OK;
    }
    if (op.k_in() > kInlineSrc || op.m_out() > kInlineDst) return run_ptr_batch(op, {blocks}, B, st);
    int status = ECG_OK;
    std::shared_ptr<ProgramSet> ps = program_set(&op, 1, &status, st);
    if (!ps) return status;
    if (const int rc = ps->ensure_ready(st); rc != ECG_OK) return rc;
    GfLaunch a;
    memset(&a, 0, sizeof(a));
    a.tabs = ps->d_tabs;
    a.src_ids = ps->d_src;
    a.dst_ids = ps->d_dst;
    a.B = B;
    a.k = ps->k;
    a.m = ps->m;
    a.S = 1;
    a.MT = ps->MT;
    a.rtiles = ps->rtiles;
    a.binary = ps->binary ? 1 : 0;
    bool vec_ok = true;
    for (int d : op.dst_ids) vec_ok &= aligned16(blocks[d]);
    for (int s : op.src_ids) vec_ok &= aligned16(blocks[s]);
    for (int j = 0; j < op.k_in(); j++) a.isrc[j] = blocks[op.src_ids[j]];
    for (int p = 0; p < op.m_out(); p++) a.idst[p] = blocks[op.dst_ids[p]];
    a.done_flags = latency ? flags : nullptr;
    a.done_seq = seq;
    // A single small call fills a few dozen workgroups: its time is the latency chain, not bandwidth, so
    // small blocks take the latency kernel (every load in flight at once) on the device tier as well.
    const bool lat = latency || (B <= get_option(ECG_OPT_LAT_DWORD_BYTES) && op.k_in() <= kLatMaxSrc);
    ECG_HIP(launch_gf(a, lat ? GF_MODE_INLINE_LAT : GF_MODE_INLINE, vec_ok, st, n_flags));
    if (!host_tier) note_launch(*ps, st);
    return ECG_OK;
}

// ------------------------------------------------------------------------------------------------
// Deferred-batch scope (engine.hpp).

namespace {

struct DeferScope {
    bool active = false;
    std::vector<DeferredCall> q;
    ScratchRanges scratch;
    FlushStats stats;
    // the stream and device of the last group the scope launched: a scope flushes several times (every
    // kEagerFlush calls, before a host-tier call, on ecg_batch_flush), and the first group of a flush must
    // wait for the previous flush's last group when it runs on another stream.  That stream is compared,
    // never named: the caller may have destroyed it since (profiles/r04/stream/), so a flush that leaves the
    // scope open records the ordering event behind its last group before it returns (last_recorded).
    hipStream_t last_st = nullptr;
    int last_dev = -1;
    bool last_recorded = false;
    // ordering events, one per device the scope launched on, leased from that device's engine pool for the
    // scope and returned at its end (or at thread exit): none is held per thread between scopes
    std::vector<std::pair<Engine*, hipEvent_t>> order_evs;
    hipEvent_t order_ev(int dev) {
        for (auto& e : order_evs)
            if (e.first->device() == dev) return e.second;
        return nullptr;
    }
    void release_order_evs() {
        for (auto& e : order_evs) e.first->release_event(e.second);
        order_evs.clear();
    }
    // Deferred HOST-tier calls (ecg_batch_defer_host): a call's input blocks are copied into the pinned
    // staging of a host context leased for the scope when the call is made (region A, one slot per block
    // read before written); its outputs get slots in region W and reach the caller's buffers at the flush.
    // The flush moves region A in ONE H2D copy, launches the calls grouped by plan, moves W back in ONE D2H
    // copy and scatters it -- the synchronous per-call round trip (launch + completion + two copies) is paid
    // once per flush instead of once per call.  At most one of the two queues (device-tier q, host-tier hq)
    // holds calls at any time: recording into one flushes the other first.
    bool host_defer = false;
    struct HostCall {
        Engine* eng;
        std::shared_ptr<const std::vector<LinearOp>> ops;
        std::vector<uint8_t*> host;  // the caller's block pointers
        std::vector<int> slot;       // >= 0: region-A slot; <= -2: region-W slot -2 - slot; -1: unused
        std::vector<int> wr;         // block ids the call writes
    };
    std::vector<HostCall> hq;
    int h_up = 0, h_w = 0;
    long long h_B = -1;
    bool h_inplace = false;  // a written block has a region-A slot (read, then written)
    PtrGroups h_out;         // pending output blocks by B-byte bucket (pending_output_overlaps), open addressing
    size_t h_nout = 0;       // entries in h_out (a block is written at most once per batch: a second write flushes)
    std::unique_ptr<CtxLease> h_ctx;
    ~DeferScope() { release_order_evs(); }
};

thread_local DeferScope t_defer;
constexpr size_t kMaxDeferred = 1 << 16;  // calls recorded before an automatic flush
// Without declared scratch, a flush of the calls recorded so far changes nothing but where groups are
// cut, so the scope flushes every kEagerFlush calls: the GPU runs the first calls while the host records
// the rest, instead of idling until the scope ends.  (With scratch, a flush would write pending scratch
// contents for real; such scopes flush only at kMaxDeferred.)
constexpr size_t kEagerFlush = 1024;

size_t flush_at() { return t_defer.scratch.empty() ? kEagerFlush : kMaxDeferred; }

bool same_ops(const std::vector<LinearOp>& a, const std::vector<LinearOp>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); i++)
        if (a[i].src_ids != b[i].src_ids || a[i].dst_ids != b[i].dst_ids || a[i].coef != b[i].coef) return false;
    return true;
}

// Pointer tables for pointer-table launches: a per-device ring of pinned host + device slots shared by
// all threads (process lifetime, so no per-thread leak), each slot locked while it is filled and its
// launch enqueued, and reused only after that launch has completed (its event).
struct TableSlot {
    std::mutex mu;
    void* host = nullptr;
    void* dev = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    hipEvent_t up_ev = nullptr;  // the upload's completion, on the upload stream (upload_table)
    bool pending = false;
};
constexpr int kTableSlots = 16;
TableSlot g_tables[kMaxDevices][kTableSlots];
std::atomic<unsigned> g_table_next[kMaxDevices];

// Pointer tables go to the device ahead of the launch that reads them.  On the launch's own stream the copy
// waits for every earlier kernel there and the launch then waits for the copy: a DMA round trip between two
// kernels.  ECG_TABLE_UPLOAD=1 puts the copy on a per-device upload stream instead, so it runs while the launch
// stream's earlier kernels do, and the launch waits for it through an event (A/B switch, read once).  The slot's
// memory is rewritten only after its previous launch completed (TableSlot::ev), which waited for its upload.
bool table_upload_stream() {
    static const bool on = getenv("ECG_TABLE_UPLOAD") && atoi(getenv("ECG_TABLE_UPLOAD")) == 1;
    return on;
}
std::mutex g_upload_mu;
hipStream_t g_upload_stream[kMaxDevices];

hipError_t upload_table(int dev, TableSlot& t, size_t bytes, hipStream_t st) {
    if (!table_upload_stream()) return hipMemcpyAsync(t.dev, t.host, bytes, hipMemcpyHostToDevice, st);
    hipStream_t u;
    {
        std::lock_guard<std::mutex> lk(g_upload_mu);
        if (!g_upload_stream[dev]) {
            const hipError_t e = hipStreamCreateWithFlags(&g_upload_stream[dev], hipStreamNonBlocking);
            if (e != hipSuccess) return e;
        }
        u = g_upload_stream[dev];
    }
    hipError_t e;
    if (!t.up_ev && (e = hipEventCreateWithFlags(&t.up_ev, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(t.dev, t.host, bytes, hipMemcpyHostToDevice, u)) != hipSuccess) return e;
    if ((e = hipEventRecord(t.up_ev, u)) != hipSuccess) {
        (void)hipStreamSynchronize(u);
        return e;
    }
    return hipStreamWaitEvent(st, t.up_ev, 0);
}

// One side (the inputs or the outputs of `ids`) of a run of recorded calls in the strided form
// base + call * sstride + v[j] * bstride.  True only if EVERY pointer of every call is exactly that, so
// a strided launch touches exactly the bytes the pointer-table launch would.  A per-stripe loop over
// one [S][n][B] batch in HBM (the reference's proxy loop on device buffers) has this form.
bool strided_side(const std::vector<const uint8_t* const*>& calls, const std::vector<int>& ids,
                  const uint8_t*& base, long long& sstride, long long& bstride, std::vector<int>& v) {
    const size_t R = calls.size(), n = ids.size();
    if (R < 2 || n == 0) return false;
    uintptr_t lo = UINTPTR_MAX;
    for (int id : ids) lo = std::min(lo, (uintptr_t)calls[0][id]);
    unsigned long long g = 0;
    for (int id : ids) g = std::gcd(g, (unsigned long long)((uintptr_t)calls[0][id] - lo));
    v.resize(n);
    for (size_t j = 0; j < n; j++) {
        const unsigned long long q = g ? ((uintptr_t)calls[0][ids[j]] - lo) / g : 0;
        if (q > 0x7fffffffULL) return false;
        v[j] = (int)q;
    }
    const uintptr_t p00 = (uintptr_t)calls[0][ids[0]], p10 = (uintptr_t)calls[1][ids[0]];
    if (p10 <= p00 || p10 - p00 > (uintptr_t)(1ULL << 40)) return false;
    const uintptr_t st = p10 - p00;
    for (size_t c = 0; c < R; c++)
        for (size_t j = 0; j < n; j++)
            if ((uintptr_t)calls[c][ids[j]] != (uintptr_t)calls[0][ids[j]] + c * st) return false;
    base = (const uint8_t*)lo;
    sstride = (long long)st;
    bstride = (long long)g;
    return true;
}

// Fast path of a flush: every recorded call has the same plan (one interned object), stream, engine and
// block size, and the blocks of all calls form one strided batch in which no two (call, block) pairs
// overlap -- a per-stripe loop over one [S][n][B] batch, or over a block-major [n][S][B] one.  Then no call
// reads or writes a block another call touches, so they form ONE group: what schedule_groups would
// return, without hashing every block address.  Overlap-free when either
//   (a) blocks of a call are >= B apart and whole stripes are apart: ss >= (vmax - vmin) * bs + B, or
//   (b) calls are >= B apart and whole block rows are apart: bs >= (R - 1) * ss + B.
bool one_disjoint_strided_group(const std::vector<DeferredCall>& q) {
    const size_t R = q.size();
    if (R < 2) return false;
    const DeferredCall& a = q[0];
    for (const DeferredCall& c : q)
        if (c.ops.get() != a.ops.get() || c.st != a.st || c.B != a.B || c.eng != a.eng) return false;
    thread_local std::vector<int> ids, v;
    thread_local std::vector<const uint8_t* const*> calls;
    ids.clear();
    for (const LinearOp& op : *a.ops) {
        ids.insert(ids.end(), op.src_ids.begin(), op.src_ids.end());
        ids.insert(ids.end(), op.dst_ids.begin(), op.dst_ids.end());
    }
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    calls.resize(R);
    for (size_t c = 0; c < R; c++) calls[c] = q[c].blocks.data();
    const uint8_t* base = nullptr;
    long long ss = 0, bs = 0;
    if (!strided_side(calls, ids, base, ss, bs, v)) return false;
    const long long B = a.B;
    const int vmin = *std::min_element(v.begin(), v.end()), vmax = *std::max_element(v.begin(), v.end());
    if (vmax == vmin) return ss >= B;  // one block per call (or every id the same block)
    if (bs < B) return false;
    return ss >= (long long)(vmax - vmin) * bs + B || (ss >= B && bs >= (long long)(R - 1) * ss + B);
}

}  // namespace

// A run of recorded calls whose blocks form one strided batch goes out as a strided launch (the
// batched tier's kernel: no pointer table, 10-15 % less kernel time on the config-2 batch); any other
// run keeps the pointer-table launch.  *done = false: not strided, nothing launched.
int Engine::run_calls_strided(const LinearOp& op, const std::vector<const uint8_t* const*>& calls, long long B,
                              hipStream_t st, bool* done) {
    *done = false;
    const uint8_t *ib = nullptr, *ob = nullptr;
    long long iss = 0, ibs = 0, oss = 0, obs = 0;
    std::vector<int> vi, vo;
    if (!strided_side(calls, op.src_ids, ib, iss, ibs, vi) || !strided_side(calls, op.dst_ids, ob, oss, obs, vo))
        return ECG_OK;
    if ((((uintptr_t)ib | (uintptr_t)ob) & 15) || ((iss | ibs | oss | obs) & 15)) return ECG_OK;
    LinearOp s2 = op;
    s2.src_ids = vi;
    s2.dst_ids = vo;
    *done = true;
    return run_strided({s2}, nullptr, (int)calls.size(), ib, iss, ibs, (void*)ob, oss, obs, B, st);
}

bool batch_active() { return t_defer.active; }

int batch_begin() {
    if (t_defer.active) return ECG_EINVAL;  // scopes do not nest
    t_defer.active = true;
    t_defer.q.clear();
    t_defer.scratch.clear();
    t_defer.last_st = nullptr;
    t_defer.last_dev = -1;
    t_defer.last_recorded = false;
    t_defer.host_defer = false;
    return ECG_OK;
}

int batch_defer_host(int on) {
    if (!t_defer.active) return ECG_EINVAL;
    if (!on && !t_defer.hq.empty()) {
        const int rc = host_flush();
        if (rc != ECG_OK) return rc;
    }
    t_defer.host_defer = on != 0;
    return ECG_OK;
}

int batch_scratch(const void* p, size_t bytes) {
    if (!t_defer.active || !p) return ECG_EINVAL;
    if (bytes == 0) return ECG_OK;
    if ((uintptr_t)p + bytes < (uintptr_t)p) return ECG_EINVAL;
    t_defer.scratch.add((uintptr_t)p, (uintptr_t)p + bytes);
    return ECG_OK;
}

FlushStats last_flush_stats() { return t_defer.stats; }

// ScratchRanges: sorted disjoint [lo, hi); add() merges overlapping and touching ranges.
void ScratchRanges::add(uintptr_t lo, uintptr_t hi) {
    auto it = std::lower_bound(r_.begin(), r_.end(), std::make_pair(lo, (uintptr_t)0));
    if (it != r_.begin() && std::prev(it)->second >= lo) --it;
    auto e = it;
    while (e != r_.end() && e->first <= hi) {
        lo = std::min(lo, e->first);
        hi = std::max(hi, e->second);
        ++e;
    }
    it = r_.erase(it, e);
    r_.insert(it, {lo, hi});
}

bool ScratchRanges::holds(const void* p, long long B) const {
    const uintptr_t a = (uintptr_t)p;
    auto it = std::upper_bound(r_.begin(), r_.end(), std::make_pair(a, UINTPTR_MAX));
    if (it == r_.begin()) return false;
    --it;
    return a >= it->first && a + (uintptr_t)B <= it->second;
}

namespace {

// A linear combination of real blocks over GF(2^8): (block, coefficient) terms, coefficients != 0 once
// normalised.  Small (a partial repair combines <= k' blocks), so a flat vector.
using Term = std::pair<uint8_t*, uint8_t>;
using Terms = std::vector<Term>;

void add_term(Terms& t, uint8_t* p, int c) {
    if (!c) return;
    for (auto& x : t)
        if (x.first == p) {
            x.second ^= (uint8_t)c;
            return;
        }
    t.emplace_back(p, (uint8_t)c);
}

void drop_zero_terms(Terms& t) {
    t.erase(std::remove_if(t.begin(), t.end(), [](const Term& x) { return x.second == 0; }), t.end());
}

// Open-addressing map block address -> int, -1 = absent.  Entries are never erased (set to -1): one flush
// touches few distinct addresses, and the map lives for one flush.
class PtrInt {
public:
    int get(const void* ptr) const {
        if (slots_.empty()) return -1;
        const uintptr_t p = (uintptr_t)ptr;
        for (size_t i = hash(p) & mask_;; i = (i + 1) & mask_) {
            if (slots_[i].p == p) return slots_[i].v;
            if (slots_[i].p == 0) return -1;
        }
    }
    int& ref(const void* ptr) {
        if ((count_ + 1) * 2 > slots_.size()) grow();
        const uintptr_t p = (uintptr_t)ptr;
        for (size_t i = hash(p) & mask_;; i = (i + 1) & mask_) {
            if (slots_[i].p == p) return slots_[i].v;
            if (slots_[i].p == 0) {
                slots_[i] = Slot{p, -1};
                count_++;
                return slots_[i].v;
            }
        }
    }
    // empty, with room for n addresses without growing
    void reset(size_t n) {
        size_t want = 256;
        while (want < 4 * n) want <<= 1;
        if (slots_.size() < want) {
            slots_.assign(want, Slot{0, -1});
            mask_ = want - 1;
        } else if (count_) {
            std::fill(slots_.begin(), slots_.end(), Slot{0, -1});
        }
        count_ = 0;
    }
    template <class F>
    void for_each(F f) const {
        for (const Slot& s : slots_)
            if (s.p && s.v >= 0) f((uint8_t*)s.p, s.v);
    }

private:
    struct Slot {
        uintptr_t p;
        int v;
    };
    static size_t hash(uintptr_t p) { return ptr_hash(p); }
    void grow() {
        std::vector<Slot> old;
        old.swap(slots_);
        slots_.assign(old.empty() ? 256 : old.size() * 2, Slot{0, -1});
        mask_ = slots_.size() - 1;
        count_ = 0;
        for (const Slot& s : old)
            if (s.p) ref((const void*)s.p) = s.v;
    }
    std::vector<Slot> slots_;
    size_t mask_ = 0, count_ = 0;
};

// compose_scratch's state (engine.hpp).  Expressions live in a slab indexed from `ex_`; `users_` maps a
// real block to a list of (expression, generation) nodes that read it -- a node whose generation is no
// longer its slot's is stale.  Composed plans are interned by content, so the flush's plan classes see
// one plan pointer per distinct composed map.
class Composer {
public:
    std::vector<DeferredCall> out;
    long long nmat = 0;

    // One Composer per thread, reused by every flush (its tables and buffers keep their capacity).
    void reset(const ScratchRanges& s, size_t ncalls) {
        scratch_ = &s;
        out.clear();
        out.reserve(ncalls);
        nmat = 0;
        slab_used_ = 0;
        free_.clear();
        uses_.clear();
        ex_.reset(ncalls);
        users_.reset(4 * ncalls);
        if (plans_.size() > 4096) plans_.clear();  // interned composed plans: bounded
    }

    void call(DeferredCall&& c) {
        bool touches = false;
        for (const LinearOp& op : *c.ops) {
            for (int id : op.src_ids) touches = touches || ex_.get(c.blocks[id]) >= 0;
            for (int id : op.dst_ids) touches = touches || scratch_->holds(c.blocks[id], c.B);
        }
        if (!touches) {
            // expressions reading blocks this call overwrites go out first, together as one op
            if (!uses_.empty()) {
                fast_.clear();
                start_collect(&fast_, c.eng, c.B);
                for (const LinearOp& op : *c.ops)
                    for (int id : op.dst_ids) before_write(c.blocks[id]);
                collect_ = nullptr;
                if (fast_.n) emit(c.eng, c.st, c.B, fast_);
            }
            out.push_back(std::move(c));
            return;
        }
        for (const LinearOp& op : *c.ops) one_op(c, op);
    }

    void finish(bool scope_end) {
        if (scope_end) return;  // unconsumed scratch contents are undefined after the scope
        std::vector<uint8_t*> left;  // a mid-scope flush leaves memory as the sequential calls would
        ex_.for_each([&](uint8_t* p, int) { left.push_back(p); });
        std::sort(left.begin(), left.end());
        write_out(left);
    }

private:
    struct Expr {
        Engine* eng;
        hipStream_t st;
        long long B;
        uint8_t* self;
        uint32_t gen;
        Terms t;
    };
    struct Use {
        int expr;
        uint32_t gen;
        int next;
    };
    // rows (block, terms) of one op being built; elements keep their capacity across uses
    struct RowBuf {
        std::vector<std::pair<uint8_t*, Terms>> v;
        size_t n = 0;
        void clear() { n = 0; }
        Terms& add(uint8_t* d) {
            if (n == v.size()) v.emplace_back();
            v[n].first = d;
            return v[n++].second;
        }
    };

    void one_op(const DeferredCall& c, const LinearOp& op) {
        const int k = op.k_in(), m = op.m_out();
        // inputs whose expression was recorded on another stream / device / block size are written for
        // real first -- before any row is built, since writing them out can overwrite blocks other
        // expressions (and so the rows) read
        std::vector<uint8_t*> foreign;
        for (int id : op.src_ids) {
            const int e = ex_.get(c.blocks[id]);
            if (e >= 0 && !(slab_[e].eng == c.eng && slab_[e].st == c.st && slab_[e].B == c.B))
                foreign.push_back(c.blocks[id]);
        }
        if (!foreign.empty()) write_out(foreign);
        if ((int)rows_.size() < m) rows_.resize((size_t)m);
        for (int p = 0; p < m; p++) {
            Terms& t = rows_[p];
            t.clear();
            for (int j = 0; j < k; j++) {
                const int cf = op.coef[(size_t)p * k + j];
                if (!cf) continue;
                uint8_t* src = c.blocks[op.src_ids[j]];
                const int e = ex_.get(src);
                if (e >= 0) {
                    for (const Term& x : slab_[e].t) add_term(t, x.first, gf::mul(cf, x.second));
                    continue;
                }
                add_term(t, src, cf);
            }
            drop_zero_terms(t);
        }
        // virtual writes first: a new expression may read a block this same op overwrites, and the real
        // writes below then write it out (into this op) like any other expression reading it.  A virtual
        // write leaves d's memory as it is, so expressions reading the real d stay valid.
        for (int p = 0; p < m; p++) {
            uint8_t* d = c.blocks[op.dst_ids[p]];
            if (!scratch_->holds(d, c.B)) continue;
            int& slot = ex_.ref(d);
            if (slot < 0) {
                if (!free_.empty()) {
                    slot = free_.back();
                    free_.pop_back();
                } else {
                    if (slab_used_ == slab_.size()) slab_.emplace_back();
                    slot = (int)slab_used_++;
                }
            }
            const int e = slot;
            Expr& x = slab_[e];
            x.eng = c.eng;
            x.st = c.st;
            x.B = c.B;
            x.self = d;
            x.gen = ++gen_;
            x.t.assign(rows_[p].begin(), rows_[p].end());
            for (const Term& u : x.t) {
                int& head = users_.ref(u.first);
                uses_.push_back(Use{e, x.gen, head});
                head = (int)uses_.size() - 1;
            }
        }
        real_.clear();
        start_collect(&real_, c.eng, c.B);
        for (int p = 0; p < m; p++) {
            uint8_t* d = c.blocks[op.dst_ids[p]];
            if (scratch_->holds(d, c.B)) continue;
            before_write(d);
            real_.add(d).assign(rows_[p].begin(), rows_[p].end());
        }
        collect_ = nullptr;
        if (real_.n) emit(c.eng, c.st, c.B, real_);
    }

    // While a call's writes are processed, expressions written out because the call overwrites a block
    // they read join the call's own op (`collect_`): one op reads every input before it writes any
    // output, so neither side sees the other's writes (a separate earlier call writing scratch block s
    // would clobber an s the op itself still reads).  An expression recorded on another stream of the same
    // device joins too: the flush orders its groups across streams (batch_flush), so the op is ordered
    // after the other stream's writes to the blocks the expression reads.  Written out on its own stream
    // instead, it would break the op's read-before-write when the two read each other's blocks (the
    // sequential interpreter of tests/sanitize/host_fuzz.cpp finds such cycles).
    void start_collect(RowBuf* rows, Engine* eng, long long B) {
        collect_ = rows;
        ceng_ = eng;
        cB_ = B;
    }

    void materialise(uint8_t* s) {
        int& slot = ex_.ref(s);
        if (slot < 0) return;
        const int e = slot;
        slot = -1;
        Expr& x = slab_[e];
        const Engine* eng = x.eng;
        Engine* eng_mut = x.eng;
        hipStream_t st = x.st;
        const long long B = x.B;
        Terms t;
        t.swap(x.t);
        x.gen = ++gen_;  // every node still naming this slot is stale now
        free_.push_back(e);
        before_write(s);
        if (collect_ && eng == ceng_ && B == cB_) {
            collect_->add(s).swap(t);
        } else {
            RowBuf one;
            one.add(s).swap(t);
            emit(eng_mut, st, B, one);
        }
        nmat++;
    }

    // Top level: write the expressions of `ss` out, with every expression they drag along, as ONE op
    // (expressions can read each other's real blocks both ways once a scratch block's expression read
    // its own old contents, so written one by one the second would read the first's new bytes).
    void write_out(const std::vector<uint8_t*>& ss) {
        RowBuf& rows = wo_;
        rows.clear();
        Engine* eng = nullptr;
        hipStream_t st = nullptr;
        long long B = 0;
        for (uint8_t* s : ss) {
            const int e = ex_.get(s);
            if (e < 0) continue;
            if (!collect_) {
                eng = slab_[e].eng;
                st = slab_[e].st;
                B = slab_[e].B;
                start_collect(&rows, eng, B);
            }
            materialise(s);
        }
        collect_ = nullptr;
        if (rows.n) emit(eng, st, B, rows);
    }

    // d is about to be overwritten: every expression still reading d is written out first
    void before_write(uint8_t* d) {
        if (uses_.empty()) return;
        const int h = users_.get(d);
        if (h < 0) return;
        users_.ref(d) = -1;
        for (int u = h; u >= 0; u = uses_[u].next) {
            const Use nd = uses_[u];
            Expr& x = slab_[nd.expr];
            if (x.gen != nd.gen) continue;  // stale: the slot was rewritten or written out since
            for (const Term& t : x.t)
                if (t.first == d) {
                    materialise(x.self);
                    break;
                }
        }
    }

    // One composed call writing rows[i].first = rows[i].second: inputs in first-appearance order (the same
    // for every stripe of one call pattern, so equal patterns intern to one plan), rows that combine to
    // nothing become a k_in = 0 op (zero bytes, what the sequential calls leave there).  A block written
    // twice by one op holds its last row (every row reads before any row writes).
    void emit(Engine* eng, hipStream_t st, long long B, const RowBuf& buf) {
        DeferredCall c{eng, st, B, nullptr, {}};
        const std::pair<uint8_t*, Terms>* rows = buf.v.data();
        const size_t nrows = buf.n;
        keep_.assign(nrows, 1);
        for (size_t i = 0; i < nrows; i++)
            for (size_t j = i + 1; j < nrows && keep_[i]; j++)
                if (rows[j].first == rows[i].first) keep_[i] = 0;
        ins_.clear();
        for (size_t i = 0; i < nrows; i++)
            if (keep_[i])
                for (const Term& x : rows[i].second)
                    if (std::find(ins_.begin(), ins_.end(), x.first) == ins_.end()) ins_.push_back(x.first);
        const int n = (int)ins_.size();
        // content key: n, then per kept row a zero flag or its n coefficients
        key_.assign((const uint8_t*)&n, (const uint8_t*)&n + sizeof n);
        c.blocks.reserve(ins_.size() + nrows);
        c.blocks.assign(ins_.begin(), ins_.end());
        for (size_t i = 0; i < nrows; i++) {
            if (!keep_[i]) continue;
            c.blocks.push_back(rows[i].first);
            key_.push_back(rows[i].second.empty() ? 0 : 1);
            if (rows[i].second.empty()) continue;
            const size_t base = key_.size();
            key_.resize(base + (size_t)n, 0);
            for (const Term& x : rows[i].second)
                key_[base + (size_t)(std::find(ins_.begin(), ins_.end(), x.first) - ins_.begin())] = x.second;
        }
        uint64_t h = 1469598103934665603ull;
        for (uint8_t b : key_) h = (h ^ b) * 1099511628211ull;
        auto& bucket = plans_[h];
        for (auto& pl : bucket)
            if (pl.first == key_) {
                c.ops = pl.second;
                out.push_back(std::move(c));
                return;
            }
        auto ops = std::make_shared<std::vector<LinearOp>>();
        LinearOp full, zero;
        for (int j = 0; j < n; j++) full.src_ids.push_back(j);
        int id = n;
        size_t at = sizeof n;
        for (size_t i = 0; i < nrows; i++) {
            if (!keep_[i]) continue;
            const bool nz = key_[at++];
            if (!nz) {
                zero.dst_ids.push_back(id++);
                continue;
            }
            full.dst_ids.push_back(id++);
            full.coef.insert(full.coef.end(), key_.begin() + (long)at, key_.begin() + (long)at + n);
            at += (size_t)n;
        }
        if (full.m_out() > 0) ops->push_back(std::move(full));
        if (zero.m_out() > 0) ops->push_back(std::move(zero));
        c.ops = ops;
        bucket.emplace_back(key_, std::move(ops));
        out.push_back(std::move(c));
    }

    const ScratchRanges* scratch_ = nullptr;
    std::vector<Expr> slab_;
    size_t slab_used_ = 0;
    std::vector<int> free_;
    PtrInt ex_, users_;
    std::vector<Use> uses_;
    uint32_t gen_ = 0;
    RowBuf* collect_ = nullptr;
    RowBuf real_, fast_, wo_;
    const Engine* ceng_ = nullptr;
    long long cB_ = 0;
    std::vector<Terms> rows_;
    std::vector<uint8_t*> ins_;
    std::vector<char> keep_;
    std::vector<uint8_t> key_;
    std::unordered_map<uint64_t, std::vector<std::pair<std::vector<uint8_t>, std::shared_ptr<const std::vector<LinearOp>>>>>
        plans_;
};

}  // namespace

std::vector<DeferredCall> compose_scratch(std::vector<DeferredCall>&& q, const ScratchRanges& scratch, bool scope_end,
                                          long long* materialised) {
    thread_local Composer cp;
    cp.reset(scratch, q.size());
    for (DeferredCall& c : q) cp.call(std::move(c));
    cp.finish(scope_end);
    if (materialised) *materialised = cp.nmat;
    std::vector<DeferredCall> out;
    out.swap(cp.out);
    return out;
}

namespace {

// Plan classes of a flush: calls with equal plans (by content), block size, stream and device share a
// class.  Recording shares the plan pointer between consecutive equal calls, so most lookups hit the
// pointer cache; composed calls are interned by content.  Single-op plans of one shape (k_in, m_out) share a
// class whatever their coefficients: the per-stripe repairs of a batch (a pattern per stripe, each composing
// to its own matrix) then go out as ONE multi-program pointer-table launch per scope instead of a launch per
// pattern (families workload: RS(12,4) repairs 16 patterns x 4 scopes -> 4 launches).
class PlanClasses {
public:
    int plan_of_last() const { return last_plan_; }
    int of(const DeferredCall& c) {
        auto pk = by_ptr_.find(c.ops.get());
        int plan;
        if (pk != by_ptr_.end()) {
            plan = pk->second;
        } else {
            size_t h = 1469598103934665603ull;
            auto mix = [&](const void* p, size_t n) {
                const uint8_t* b = (const uint8_t*)p;
                for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
            };
            for (const LinearOp& op : *c.ops) {
                mix(op.src_ids.data(), op.src_ids.size() * 4);
                mix(op.dst_ids.data(), op.dst_ids.size() * 4);
                mix(op.coef.data(), op.coef.size());
                mix("|", 1);
            }
            plan = -1;
            for (int id : by_hash_[h])
                if (same_ops(*plans_[id], *c.ops)) plan = id;
            if (plan < 0) {
                plan = (int)plans_.size();
                plans_.push_back(c.ops);
                by_hash_[h].push_back(plan);
            }
            by_ptr_[c.ops.get()] = plan;
        }
        last_plan_ = plan;
        int cls_plan = plan;
        if (c.ops->size() == 1 && (*c.ops)[0].k_in() > 0) {
            const auto sk = std::make_pair((*c.ops)[0].k_in(), (*c.ops)[0].m_out());
            auto si = shapes_.find(sk);
            if (si == shapes_.end()) si = shapes_.emplace(sk, (int)shapes_.size()).first;
            cls_plan = -1 - si->second;
        }
        const auto key = std::make_tuple(cls_plan, c.eng, c.st, c.B);
        auto it = cls_.find(key);
        if (it != cls_.end()) return it->second;
        const int id = (int)cls_.size();
        cls_.emplace(key, id);
        return id;
    }

private:
    std::unordered_map<const void*, int> by_ptr_;
    std::unordered_map<size_t, std::vector<int>> by_hash_;
    std::vector<std::shared_ptr<const std::vector<LinearOp>>> plans_;
    std::map<std::pair<int, int>, int> shapes_;
    std::map<std::tuple<int, Engine*, hipStream_t, long long>, int> cls_;
    int last_plan_ = -1;
};

}  // namespace

// Record the scope's ordering event of device `dev` (the current device) behind the work enqueued on `st` so
// far; `st` is a stream of the flush in progress, alive for the duration of the call.
int order_after(hipStream_t st, int dev) {
    if (dev < 0 || dev >= kMaxDevices) return ECG_EINVAL;
    DeferScope& d = t_defer;
    hipEvent_t ev = d.order_ev(dev);
    if (!ev) {
        Engine& eng = Engine::instance();  // the engine of the current device, dev
        if (!(ev = eng.acquire_event())) {
            set_last_error("batch flush: hipEventCreate failed");
            return ECG_EHIP;
        }
        d.order_evs.emplace_back(&eng, ev);
    }
    if (hipEventRecord(ev, st) != hipSuccess) {
        set_last_error("batch flush: hipEventRecord failed");
        return ECG_EHIP;
    }
    return ECG_OK;
}

int batch_flush() {
    DeferScope& d = t_defer;
    if (d.q.empty()) return ECG_OK;
    std::vector<DeferredCall> q;
    q.swap(d.q);
    FlushStats st;
    st.recorded = (long long)q.size();
    if (!d.scratch.empty()) q = compose_scratch(std::move(q), d.scratch, /*scope_end=*/!d.active, &st.materialised);
    st.composed = (long long)q.size();
    std::vector<std::vector<size_t>> groups;
    std::vector<int> plan_id;  // per call: its plan (by content); empty on the fast path (one plan)
    if (d.scratch.empty() && one_disjoint_strided_group(q)) {  // the per-stripe loop over one batch
        groups.emplace_back(q.size());
        std::iota(groups[0].begin(), groups[0].end(), (size_t)0);
    } else {
        PlanClasses classes;
        std::vector<int> cls(q.size());
        plan_id.resize(q.size());
        for (size_t c = 0; c < q.size(); c++) {
            cls[c] = classes.of(q[c]);
            plan_id[c] = classes.plan_of_last();
        }
        auto reads = [&](size_t c, auto&& f) {
            for (const LinearOp& op : *q[c].ops)
                for (int id : op.src_ids) f(q[c].blocks[id]);
        };
        auto writes = [&](size_t c, auto&& f) {
            for (const LinearOp& op : *q[c].ops)
                for (int id : op.dst_ids) f(q[c].blocks[id]);
        };
        groups = schedule_groups(q.size(), [&](size_t c) { return cls[c]; }, reads, writes);
    }
    st.groups = (long long)groups.size();
    int caller_dev = -1, cur_dev = -1;
    (void)hipGetDevice(&caller_dev);
    cur_dev = caller_dev;
    int rc = ECG_OK;
    // the previous group: the last one of the scope's previous flush, if any (its ordering event is then
    // already recorded: that flush's stream is not named again)
    hipStream_t prev_st = d.last_st;
    int prev_dev = d.last_dev;
    bool prev_recorded = d.last_recorded;
    auto set_dev = [&](int dev) {
        if (dev == cur_dev) return ECG_OK;
        if (hipSetDevice(dev) != hipSuccess) {
            set_last_error("batch flush: hipSetDevice failed");
            return ECG_EHIP;
        }
        cur_dev = dev;
        return ECG_OK;
    };
    for (size_t g = 0; g < groups.size() && rc == ECG_OK; g++) {
        const std::vector<size_t>& G = groups[g];
        const DeferredCall& c0 = q[G[0]];
        Engine* eng = c0.eng;
        // Groups run in program order across streams and devices: where the stream changes from one group
        // to the next, the new stream waits for an event recorded behind the previous group (so a chain
        // A, B, A orders every group after all earlier ones).  The calls were recorded in one order; a group
        // on stream B may read blocks an earlier group on A writes, or a scratch combination recorded on A
        // (compose_scratch joins those to the op that forces them).  The chain runs across the scope's
        // flushes too: the first group of a flush follows the last group of the previous one
        // (test_batch_scope_orders_streams_across_eager_flushes).  One stream: no event at all.
        // (prev_dev, not prev_st, says whether there was a previous group: the null stream -- torch's default
        // stream -- is a stream like any other here)
        const bool switch_st = prev_dev >= 0 && (c0.st != prev_st || eng->device() != prev_dev);
        if (switch_st && !prev_recorded) {  // the event is recorded behind the previous group, on its device
            if ((rc = set_dev(prev_dev)) != ECG_OK || (rc = order_after(prev_st, prev_dev)) != ECG_OK) break;
        }
        if ((rc = set_dev(eng->device())) != ECG_OK) break;  // a group launches on its calls' device
        if (switch_st && hipStreamWaitEvent(c0.st, d.order_ev(prev_dev), 0) != hipSuccess) {
            set_last_error("batch flush: hipStreamWaitEvent failed");
            rc = ECG_EHIP;
            break;
        }
        prev_st = c0.st;
        prev_dev = eng->device();
        prev_recorded = false;
        if (G.size() == 1) {
            rc = eng->launch_direct(*c0.ops, c0.blocks.data(), c0.B, c0.st);
            st.launches += (long long)c0.ops->size();
            continue;
        }
        std::vector<const uint8_t* const*> calls;
        calls.reserve(G.size());
        for (size_t c : G) calls.push_back(q[c].blocks.data());
        bool mixed = false;  // single-op plans of one shape, several matrices (PlanClasses)
        if (!plan_id.empty())
            for (size_t c : G) mixed |= plan_id[c] != plan_id[G[0]];
        if (mixed) {
            std::vector<const LinearOp*> per_call;
            per_call.reserve(G.size());
            for (size_t c : G) per_call.push_back(&(*q[c].ops)[0]);
            rc = eng->run_ptr_batch_multi(per_call, calls, c0.B, c0.st);
            st.launches++;
            continue;
        }
        for (const LinearOp& op : *c0.ops) {
            if (op.k_in() == 0) {  // composed row of zeros: the library writes zero bytes
                for (size_t c : G) {
                    rc = eng->launch_direct({op}, q[c].blocks.data(), q[c].B, q[c].st);
                    st.launches++;
                    if (rc != ECG_OK) break;
                }
            } else {
                bool done = false;
                rc = eng->run_calls_strided(op, calls, c0.B, c0.st, &done);
                if (rc == ECG_OK && !done) rc = eng->run_ptr_batch(op, calls, c0.B, c0.st);
                st.launches++;
            }
            if (rc != ECG_OK) break;
        }
    }
    // the scope stays open: the next flush may start on another stream, so the last group's ordering event
    // is recorded now, while its stream is certainly alive (one event record per flush)
    if (rc == ECG_OK && d.active && prev_dev >= 0 && !prev_recorded) {
        if ((rc = set_dev(prev_dev)) == ECG_OK) rc = order_after(prev_st, prev_dev);
        prev_recorded = rc == ECG_OK;
    }
    if (cur_dev != caller_dev && caller_dev >= 0) (void)hipSetDevice(caller_dev);
    d.last_st = prev_st;
    d.last_dev = prev_dev;
    d.last_recorded = prev_recorded;
    d.stats = st;
    // the next recording reuses this queue's capacity (a scope of thousands of calls regrew it every flush)
    q.clear();
    if (d.q.empty() && d.q.capacity() < q.capacity()) d.q.swap(q);
    return rc;
}

int batch_flush_pending() {
    if (!t_defer.hq.empty()) return host_flush();  // at most one queue holds calls
    return t_defer.q.empty() ? ECG_OK : batch_flush();
}

int batch_flush_all() {
    const int rh = t_defer.hq.empty() ? ECG_OK : host_flush();
    const int rd = batch_flush();
    return rh != ECG_OK ? rh : rd;
}

int batch_end() {
    if (!t_defer.active) return ECG_EINVAL;
    t_defer.active = false;  // the flush below is the scope's end: unconsumed scratch is not written
    const int rh = t_defer.hq.empty() ? ECG_OK : host_flush();
    const int rd = batch_flush();
    const int rc = rh != ECG_OK ? rh : rd;
    t_defer.host_defer = false;
    t_defer.q.clear();
    t_defer.scratch.clear();
    t_defer.release_order_evs();  // a later wait on one refers to its record at the time of the wait
    return rc;
}

// ------------------------------------------------------------------------------------------------
// Deferred host-tier calls (DeferScope::hq; ecg_batch_defer_host).

namespace {

// Copy a call's input block into the scope's pinned staging with non-temporal stores.  Region A of a
// host batch grows to tens of MiB (4096 RS(6,4) 4 KiB stripes: 96 MiB), far past the caches, and ordinary
// stores pay a read-for-ownership of every destination line: the plain memcpy moved 7.8 GB/s and was most
// of a recorded call's 3.2 us (tools/defer_cost.cpp, profiles/r04/small_host/).  The flush issues an
// sfence before the H2D copy reads the region.  dst is 256-byte aligned (the slot pitch).
void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    if (((uintptr_t)dst & 15) == 0)
        for (; i + 64 <= n; i += 64) {
            const __m128i a = _mm_loadu_si128((const __m128i*)(src + i));
            const __m128i b = _mm_loadu_si128((const __m128i*)(src + i + 16));
            const __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32));
            const __m128i d = _mm_loadu_si128((const __m128i*)(src + i + 48));
            _mm_stream_si128((__m128i*)(dst + i), a);
            _mm_stream_si128((__m128i*)(dst + i + 16), b);
            _mm_stream_si128((__m128i*)(dst + i + 32), c);
            _mm_stream_si128((__m128i*)(dst + i + 48), d);
        }
    if (i < n) memcpy(dst + i, src + i, n - i);
}

constexpr size_t kHostDeferMaxBytes = 64 << 20;  // staging (regions A + W) of one host batch

// Pinned staging of the scope's context with room for `bytes`, keeping its first `keep` bytes.
int ensure_pinned(HostCtx& c, size_t bytes, size_t keep) {
    if (c.pinned_cap >= bytes) return ECG_OK;
    const size_t cap = std::max(bytes, std::max(c.pinned_cap * 2, (size_t)1 << 20));
    uint8_t* p = nullptr;
    uint8_t* pd = nullptr;
    ECG_HIP(hipHostMalloc((void**)&p, cap, hipHostMallocMapped | hipHostMallocCoherent));
    if (hipHostGetDevicePointer((void**)&pd, p, 0) != hipSuccess) {
        (void)hipHostFree(p);
        set_last_error("hipHostGetDevicePointer(host batch staging) failed");
        return ECG_EHIP;
    }
    if (keep && c.pinned) memcpy(p, c.pinned, keep);
    if (c.pinned) {
        if (c.stream) (void)hipStreamSynchronize(c.stream);
        (void)hipHostFree(c.pinned);
    }
    c.pinned = p;
    c.pinned_dev = pd;
    c.pinned_cap = cap;
    return ECG_OK;
}

void host_queue_reset() {
    DeferScope& d = t_defer;
    d.hq.clear();
    if (d.h_nout) d.h_out.reset(0);
    d.h_nout = 0;
    d.h_up = d.h_w = 0;
    d.h_B = -1;
    d.h_inplace = false;
    d.h_ctx.reset();  // a context whose batch did not complete drains its streams before its next lessee
}

// Pending outputs of the deferred host batch, compared by BYTE RANGE (host blocks of one scope
// may be offsets into one caller buffer).  Every pending output is [p, p + B) with the batch's one block
// size, and pending outputs are pairwise disjoint (a call touching one flushes first), so a B-byte bucket
// holds the start of at most one: h_out maps bucket p / B + 1 to wr = 1 and rd = p % B.  A block [a, a + B)
// overlaps a pending output iff one starts in bucket a / B - 1, a / B or a / B + 1 within B bytes of a.
void note_pending_output(DeferScope& d, const void* blk, long long B) {
    if (B <= 0) return;  // an empty block overlaps nothing
    const uintptr_t p = (uintptr_t)blk, b = (uintptr_t)B;
    PtrGroups::Slot& s = d.h_out.at((const void*)(p / b + 1));
    s.wr = 1;
    s.rd = (int)(p % b);
}

bool pending_output_overlaps(const DeferScope& d, const void* blk, long long B) {
    if (B <= 0) return false;
    const uintptr_t a = (uintptr_t)blk, b = (uintptr_t)B, q = a / b;
    for (uintptr_t k = q ? q - 1 : 0; k <= q + 1; k++) {
        const PtrGroups::Slot* s = d.h_out.find_slot((const void*)(k + 1));
        if (!s || !s->wr) continue;
        const uintptr_t p = k * b + (uintptr_t)s->rd;
        if ((p > a ? p - a : a - p) < b) return true;
    }
    return false;
}

}  // namespace

// Record one host-tier call of an open scope with host deferral on.  Returns ECG_OK (recorded), a negative
// status, or 1: not deferrable (blocks above kStagedMaxBlock, or the call alone overflows the staging) --
// the caller runs it synchronously after flushing.  A call whose blocks overlap a pending output of an
// earlier recorded call (by byte range, pending_output_overlaps), or with another block size or engine,
// flushes the batch first.
int record_host(Engine* eng, const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B) {
    DeferScope& d = t_defer;
    if (B > (long long)kStagedMaxBlock) return 1;
    thread_local std::vector<char> upload, written, used, produced;
    upload.assign(nblocks, 0);
    written.assign(nblocks, 0);
    used.assign(nblocks, 0);
    produced.assign(nblocks, 0);
    for (const LinearOp& op : ops) {
        for (int id : op.src_ids) {
            if (id < 0 || id >= nblocks || !blocks[id]) return ECG_EINVAL;
            if (!produced[id]) upload[id] = 1;
            used[id] = 1;
        }
        for (int id : op.dst_ids) {
            if (id < 0 || id >= nblocks || !blocks[id]) return ECG_EINVAL;
            produced[id] = written[id] = used[id] = 1;
        }
    }
    int nup = 0, nw = 0;
    for (int id = 0; id < nblocks; id++) {
        nup += upload[id];
        nw += used[id] && !upload[id];
    }
    const size_t pitch = ((size_t)B + 255) & ~(size_t)255;
    if ((size_t)(nup + nw) * pitch > kHostDeferMaxBytes) return 1;
    if (!d.q.empty())
        if (const int rc = batch_flush(); rc != ECG_OK) return rc;  // at most one queue holds calls
    bool flush = !d.hq.empty() && (d.h_B != B || d.hq.back().eng != eng ||
                                   (size_t)(d.h_up + d.h_w + nup + nw) * pitch > kHostDeferMaxBytes);
#ifndef ECG_TEST_NO_HOST_HAZARD_FLUSH  // test hook: a variant without this flush must fail the random-sequence test
    for (int id = 0; id < nblocks && !flush && d.h_nout; id++)
        flush = used[id] && pending_output_overlaps(d, blocks[id], B);
#endif
    if (flush)
        if (const int rc = host_flush(); rc != ECG_OK) return rc;
    if (!d.h_ctx) {
        d.h_ctx = std::make_unique<CtxLease>(eng->device());
        HostCtx& c = **d.h_ctx;
        if (!c.stream && hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess) {
            host_queue_reset();
            set_last_error("hipStreamCreate(host batch) failed");
            return ECG_EHIP;
        }
        d.h_B = B;
    }
    HostCtx& c = **d.h_ctx;
    if (const int rc = ensure_pinned(c, (size_t)(d.h_up + nup) * pitch, (size_t)d.h_up * pitch); rc != ECG_OK) {
        host_queue_reset();
        return rc;
    }
    DeferScope::HostCall call;
    call.eng = eng;
    call.host.assign(blocks, blocks + nblocks);
    call.slot.assign(nblocks, -1);
    call.wr.reserve(nblocks);
    for (int id = 0; id < nblocks; id++) {
        if (upload[id]) {
            call.slot[id] = d.h_up;
            stream_copy(c.pinned + (size_t)d.h_up * pitch, blocks[id], (size_t)B);  // inputs read at call time
            d.h_up++;
        } else if (used[id]) {
            call.slot[id] = -2 - d.h_w++;
        }
        if (written[id]) {
            call.wr.push_back(id);
            note_pending_output(d, blocks[id], B);
            d.h_nout++;
            d.h_inplace |= upload[id] != 0;
        }
    }
    if (!d.hq.empty() && same_ops(*d.hq.back().ops, ops)) call.ops = d.hq.back().ops;
    else call.ops = std::make_shared<const std::vector<LinearOp>>(ops);
    d.hq.push_back(std::move(call));
    return ECG_OK;
}

// Run the recorded host-tier calls: one H2D of region A, the calls' launches grouped by plan (consecutive
// calls with one plan: one strided or pointer-table launch per op), one D2H of region W (and of A when a
// call wrote a block it had read), then the outputs copied into the caller's buffers.  The queue is
// emptied whatever happens; on an error the outputs of this batch are undefined.
int host_flush() {
    DeferScope& d = t_defer;
    if (d.hq.empty()) return ECG_OK;
    // The batch is taken out of the scope first: the launches below go through entry points that flush
    // pending calls (run_strided), which must find nothing to flush.
    struct Batch {
        std::vector<DeferScope::HostCall> hq;
        std::unique_ptr<CtxLease> ctx;
    } bt;
    bt.hq.swap(d.hq);
    bt.ctx = std::move(d.h_ctx);
    const int h_up = d.h_up, h_w = d.h_w;
    const bool h_inplace = d.h_inplace;
    const long long B = d.h_B;
    host_queue_reset();
    HostCtx& c = **bt.ctx;
    hipStream_t st = c.stream;
    Engine* eng = bt.hq[0].eng;
    const size_t pitch = ((size_t)B + 255) & ~(size_t)255;
    const size_t a_bytes = (size_t)h_up * pitch, total = (size_t)(h_up + h_w) * pitch;
    auto fail = [&](int rc) { return rc; };  // bt's lease drains the context's streams on the way out
    int caller_dev = -1;
    (void)hipGetDevice(&caller_dev);
    const bool switched = caller_dev != eng->device() && hipSetDevice(eng->device()) == hipSuccess;
    struct Restore {
        bool on;
        int dev;
        ~Restore() {
            if (on) (void)hipSetDevice(dev);
        }
    } restore{switched, caller_dev};
    if (c.cap < total) {
        if (hipStreamSynchronize(st) != hipSuccess) return fail(ECG_EHIP);
        if (c.scratch) (void)hipFree(c.scratch);
        c.scratch = nullptr;
        c.cap = 0;
        if (hipMalloc(&c.scratch, total) != hipSuccess) {
            set_last_error("hipMalloc(host batch scratch) failed");
            return fail(ECG_EHIP);
        }
        c.cap = total;
    }
    if (const int rc = ensure_pinned(c, total, a_bytes); rc != ECG_OK) return fail(rc);
    _mm_sfence();  // the region's non-temporal stores (stream_copy) are globally visible before the DMA reads it
    if (a_bytes && hipMemcpyAsync(c.scratch, c.pinned, a_bytes, hipMemcpyHostToDevice, st) != hipSuccess) {
        set_last_error("hipMemcpyAsync(host batch H2D) failed");
        return fail(ECG_EHIP);
    }
    const size_t n = bt.hq.size();
    thread_local std::vector<uint8_t*> dptr;
    thread_local std::vector<size_t> first;
    first.resize(n + 1);
    size_t tot = 0;
    for (size_t i = 0; i < n; i++) {
        first[i] = tot;
        tot += bt.hq[i].slot.size();
    }
    first[n] = tot;
    dptr.assign(tot, nullptr);
    for (size_t i = 0; i < n; i++) {
        const auto& sl = bt.hq[i].slot;
        for (size_t id = 0; id < sl.size(); id++) {
            const int v = sl[id];
            if (v >= 0) dptr[first[i] + id] = c.scratch + (size_t)v * pitch;
            else if (v <= -2) dptr[first[i] + id] = c.scratch + a_bytes + (size_t)(-2 - v) * pitch;
        }
    }
    // Calls of one shape -- the same number of ops, and per op the same (k_in, m_out) -- form one group
    // whatever their coefficients (per-stripe decodes of different erasure patterns): the calls of a host
    // batch touch disjoint staging slots, so any grouping keeps each call's own op order.  Per op, a group
    // with one plan goes out as a strided launch (or a pointer table); mixed plans as ONE pointer-table
    // launch with a program per matrix (run_ptr_batch_multi).
    auto shape_of = [&](size_t i) {
        std::vector<int> sig;
        for (const LinearOp& op : *bt.hq[i].ops) {
            sig.push_back(op.k_in());
            sig.push_back(op.m_out());
        }
        return sig;
    };
    std::map<std::vector<int>, std::vector<size_t>> groups;
    for (size_t i = 0; i < n; i++) groups[shape_of(i)].push_back(i);
    int rc = ECG_OK;
    std::vector<const uint8_t* const*> calls;
    std::vector<const LinearOp*> per_call;
    for (auto& kv : groups) {
        const std::vector<size_t>& G = kv.second;
        if (G.size() == 1) {
            rc = eng->launch_direct(*bt.hq[G[0]].ops, dptr.data() + first[G[0]], B, st);
            if (rc != ECG_OK) break;
            continue;
        }
        calls.clear();
        for (size_t i : G) calls.push_back(dptr.data() + first[i]);
        const size_t nops = bt.hq[G[0]].ops->size();
        for (size_t o = 0; o < nops && rc == ECG_OK; o++) {
            const LinearOp& op0 = (*bt.hq[G[0]].ops)[o];
            bool one_plan = true;
            for (size_t i : G) one_plan &= bt.hq[i].ops.get() == bt.hq[G[0]].ops.get();
            if (op0.k_in() == 0) {  // composed row of zeros: the library writes zero bytes
                for (size_t i : G)
                    if (rc == ECG_OK) rc = eng->launch_direct({(*bt.hq[i].ops)[o]}, dptr.data() + first[i], B, st);
            } else if (one_plan) {
                bool done = false;
                rc = eng->run_calls_strided(op0, calls, B, st, &done);
                if (rc == ECG_OK && !done) rc = eng->run_ptr_batch(op0, calls, B, st);
            } else {
                per_call.clear();
                for (size_t i : G) per_call.push_back(&(*bt.hq[i].ops)[o]);
                rc = eng->run_ptr_batch_multi(per_call, calls, B, st);
            }
        }
        if (rc != ECG_OK) break;
    }
    if (rc != ECG_OK) return fail(rc);
    if (h_w && hipMemcpyAsync(c.pinned + a_bytes, c.scratch + a_bytes, total - a_bytes, hipMemcpyDeviceToHost, st) !=
                     hipSuccess) {
        set_last_error("hipMemcpyAsync(host batch D2H) failed");
        return fail(ECG_EHIP);
    }
    if (h_inplace && hipMemcpyAsync(c.pinned, c.scratch, a_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) {
        set_last_error("hipMemcpyAsync(host batch D2H) failed");
        return fail(ECG_EHIP);
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        set_last_error("hipStreamSynchronize(host batch) failed");
        return fail(ECG_EHIP);
    }
    for (const DeferScope::HostCall& call : bt.hq)
        for (int id : call.wr) {
            const int v = call.slot[id];
            const size_t off = v >= 0 ? (size_t)v * pitch : a_bytes + (size_t)(-2 - v) * pitch;
            memcpy(call.host[id], c.pinned + off, (size_t)B);
        }
    bt.ctx->done();
    return ECG_OK;
}

int Engine::run_ptr_batch(const LinearOp& op, const std::vector<const uint8_t* const*>& calls, long long B,
                          hipStream_t st) {
    const int S = (int)calls.size(), k = op.k_in(), m = op.m_out();
    const size_t n = (size_t)S * (k + m);
    TableSlot& t = g_tables[device_][g_table_next[device_].fetch_add(1, std::memory_order_relaxed) % kTableSlots];
    std::lock_guard<std::mutex> lk(t.mu);
    if (t.pending) {
        ECG_HIP(hipEventSynchronize(t.ev));
        t.pending = false;
    }
    if (!t.ev) ECG_HIP(hipEventCreateWithFlags(&t.ev, hipEventDisableTiming));
    if (t.cap < n * sizeof(void*)) {
        if (t.host) (void)hipHostFree(t.host);
        if (t.dev) (void)hipFree(t.dev);
        t.host = t.dev = nullptr;
        t.cap = 0;
        const size_t cap = std::max(n * sizeof(void*), (size_t)64 << 10);
        ECG_HIP(hipHostMalloc(&t.host, cap, hipHostMallocDefault));
        ECG_HIP(hipMalloc(&t.dev, cap));
        t.cap = cap;
    }
    const uint8_t** h = (const uint8_t**)t.host;
    bool aligned = true, apart = true;
    for (int s = 0; s < S; s++) {
        for (int j = 0; j < k; j++) {
            const uint8_t* p = calls[s][op.src_ids[j]];
            aligned &= aligned16(p);
            h[(size_t)s * k + j] = p;
        }
        for (int q = 0; q < m; q++) {
            const uint8_t* p = calls[s][op.dst_ids[q]];
            aligned &= aligned16(p);
            h[(size_t)S * k + (size_t)s * m + q] = p;
        }
        if (apart) apart = outputs_apart(h + (size_t)s * k, k, h + (size_t)S * k + (size_t)s * m, m, B);
    }
    ECG_HIP(upload_table(device_, t, n * sizeof(void*), st));
    const uint8_t* const* d_src = (const uint8_t* const*)t.dev;
    uint8_t* const* d_dst = (uint8_t* const*)((const uint8_t**)t.dev + (size_t)S * k);
    const int rc = run_ptrs(op, d_src, d_dst, S, B, aligned, st, apart);
    ECG_HIP(hipEventRecord(t.ev, st));
    t.pending = true;
    return rc;
}

// S calls of one op shape (k_in, m_out), call s running *ops[s] over its blocks calls[s]: ONE pointer-table
// launch with one program per distinct coefficient matrix (prog_of_stripe), instead of one launch per
// plan.  Programs are kept with canonical ids (the pointer table carries each call's own blocks), so calls
// that differ only in which blocks they name share a program.
int Engine::run_ptr_batch_multi(const std::vector<const LinearOp*>& ops, const std::vector<const uint8_t* const*>& calls,
                                long long B, hipStream_t st) {
    const int S = (int)calls.size();
    if (S == 0 || B == 0) return ECG_OK;
    if (ops.size() != calls.size()) return ECG_EINVAL;
    const int k = ops[0]->k_in(), m = ops[0]->m_out();
    if (k < 1 || m < 1) return ECG_EINVAL;
    thread_local std::vector<LinearOp> progs;
    thread_local std::vector<int> pid;
    progs.clear();
    pid.assign((size_t)S, 0);
    const LinearOp* last = nullptr;
    int last_id = -1;
    for (int c = 0; c < S; c++) {
        const LinearOp& op = *ops[c];
        if (op.k_in() != k || op.m_out() != m) return ECG_EINVAL;
        if (&op == last) {
            pid[c] = last_id;
            continue;
        }
        int id = -1;
        for (size_t p = 0; p < progs.size() && id < 0; p++)
            if (progs[p].coef == op.coef) id = (int)p;
        if (id < 0) {
            LinearOp canon;
            canon.coef = op.coef;
            for (int j = 0; j < k; j++) canon.src_ids.push_back(j);
            for (int q = 0; q < m; q++) canon.dst_ids.push_back(k + q);
            progs.push_back(std::move(canon));
            id = (int)progs.size() - 1;
        }
        pid[c] = last_id = id;
        last = &op;
    }
    if (progs.size() == 1) {  // one matrix: the plain pointer-table launch (its ids are the calls' own)
        thread_local std::vector<std::vector<const uint8_t*>> own;
        thread_local std::vector<const uint8_t* const*> rows;
        own.resize((size_t)S);
        rows.resize((size_t)S);
        for (int c = 0; c < S; c++) {
            own[c].assign((size_t)(k + m), nullptr);
            for (int j = 0; j < k; j++) own[c][j] = calls[c][ops[c]->src_ids[j]];
            for (int q = 0; q < m; q++) own[c][k + q] = calls[c][ops[c]->dst_ids[q]];
            rows[c] = own[c].data();
        }
        return run_ptr_batch(progs[0], rows, B, st);
    }
    // One set of matrices is one cache entry, whatever order the calls met them in (per-stripe
    // decodes of one batch in another order would otherwise build, and retire, a new program set each time).
    {
        thread_local std::vector<int> order, rank;
        order.resize(progs.size());
        for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
        std::sort(order.begin(), order.end(), [](int a, int b) { return progs[a].coef < progs[b].coef; });
        rank.resize(progs.size());
        bool moved = false;
        for (size_t r = 0; r < order.size(); r++) {
            rank[order[r]] = (int)r;
            moved |= order[r] != (int)r;
        }
        if (moved) {
            thread_local std::vector<LinearOp> sorted;
            sorted.clear();
            for (int i : order) sorted.push_back(std::move(progs[i]));
            progs.swap(sorted);
            for (int& x : pid) x = rank[x];
        }
    }
    int status = ECG_OK;
    std::shared_ptr<ProgramSet> ps = program_set(progs, &status, st);
    if (!ps) return status;
    if (const int rc = ps->ensure_ready(st); rc != ECG_OK) return rc;
    const size_t n = (size_t)S * (k + m);
    const size_t ptr_bytes = n * sizeof(void*), bytes = ptr_bytes + (size_t)S * sizeof(int);
    TableSlot& t = g_tables[device_][g_table_next[device_].fetch_add(1, std::memory_order_relaxed) % kTableSlots];
    std::lock_guard<std::mutex> lk(t.mu);
    if (t.pending) {
        ECG_HIP(hipEventSynchronize(t.ev));
        t.pending = false;
    }
    if (!t.ev) ECG_HIP(hipEventCreateWithFlags(&t.ev, hipEventDisableTiming));
    if (t.cap < bytes) {
        if (t.host) (void)hipHostFree(t.host);
        if (t.dev) (void)hipFree(t.dev);
        t.host = t.dev = nullptr;
        t.cap = 0;
        const size_t cap = std::max(bytes, (size_t)64 << 10);
        ECG_HIP(hipHostMalloc(&t.host, cap, hipHostMallocDefault));
        ECG_HIP(hipMalloc(&t.dev, cap));
        t.cap = cap;
    }
    const uint8_t** h = (const uint8_t**)t.host;
    int* hp = (int*)((uint8_t*)t.host + ptr_bytes);
    bool aligned = true, apart = true;
    for (int c = 0; c < S; c++) {
        const LinearOp& op = *ops[c];
        for (int j = 0; j < k; j++) {
            const uint8_t* p = calls[c][op.src_ids[j]];
            aligned &= aligned16(p);
            h[(size_t)c * k + j] = p;
        }
        for (int q = 0; q < m; q++) {
            const uint8_t* p = calls[c][op.dst_ids[q]];
            aligned &= aligned16(p);
            h[(size_t)S * k + (size_t)c * m + q] = p;
        }
        if (apart) apart = outputs_apart(h + (size_t)c * k, k, h + (size_t)S * k + (size_t)c * m, m, B);
        hp[c] = pid[c];
    }
    ECG_HIP(upload_table(device_, t, bytes, st));
    GfLaunch a;
    memset(&a, 0, sizeof(a));
    a.tabs = ps->d_tabs;
    a.src_ids = ps->d_src;
    a.dst_ids = ps->d_dst;
    a.src_ptrs = (const uint8_t* const*)t.dev;
    a.dst_ptrs = (uint8_t* const*)((const uint8_t**)t.dev + (size_t)S * k);
    a.prog_of_stripe = (const int*)((uint8_t*)t.dev + ptr_bytes);
    a.B = B;
    a.k = ps->k;
    a.m = ps->m;
    a.S = S;
    a.MT = ps->MT;
    a.rtiles = ps->rtiles;
    a.binary = ps->binary ? 1 : 0;
    a.grid_map = apart ? 2 : 0;  // the auto map's layout hint (gf_kernels.hip outputs_in_stripe)
    const hipError_t e = launch_gf(a, GF_MODE_PTRS, aligned, st);
    if (e != hipSuccess) {
        set_last_error(std::string("launch_gf(pointer table, multi): ") + hipGetErrorString(e));
        return ECG_EHIP;
    }
    note_launch(*ps, st);
    ECG_HIP(hipEventRecord(t.ev, st));
    t.pending = true;
    return ECG_OK;
}

int Engine::launch_direct(const std::vector<LinearOp>& ops, uint8_t* const* blocks, long long B, hipStream_t st) {
    for (const LinearOp& op : ops) {
        int rc = launch_one(op, blocks, B, st, /*host_tier=*/false);
        if (rc != ECG_OK) return rc;
    }
    return ECG_OK;
}

static int check_ids(const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks) {
    for (const LinearOp& op : ops) {
        for (int id : op.src_ids)
            if (id < 0 || id >= nblocks || !blocks[id]) return ECG_EINVAL;
        for (int id : op.dst_ids)
            if (id < 0 || id >= nblocks || !blocks[id]) return ECG_EINVAL;
    }
    return ECG_OK;
}

int Engine::run_device(const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B,
                       hipStream_t st) {
    if (B < 0) return ECG_EINVAL;
    if (const int rc = check_ids(ops, blocks, nblocks); rc != ECG_OK) return rc;
    if (t_defer.active) {
        if (ops.empty() || B == 0) return ECG_OK;
        if (!t_defer.hq.empty())
            if (const int rc = host_flush(); rc != ECG_OK) return rc;
        std::shared_ptr<const std::vector<LinearOp>> shared;
        if (!t_defer.q.empty() && same_ops(*t_defer.q.back().ops, ops)) shared = t_defer.q.back().ops;
        else shared = std::make_shared<const std::vector<LinearOp>>(ops);
        t_defer.q.push_back(DeferredCall{this, st, B, std::move(shared), std::vector<uint8_t*>(blocks, blocks + nblocks)});
        return t_defer.q.size() >= flush_at() ? batch_flush() : ECG_OK;
    }
    return launch_direct(ops, blocks, B, st);
}

int Engine::run_device(const std::shared_ptr<const std::vector<LinearOp>>& ops, uint8_t* const* blocks, int nblocks,
                       long long B, hipStream_t st) {
    if (B < 0 || !ops) return ECG_EINVAL;
    if (const int rc = check_ids(*ops, blocks, nblocks); rc != ECG_OK) return rc;
    if (t_defer.active) {  // recorded with the caller's (interned) plan: no copy
        if (ops->empty() || B == 0) return ECG_OK;
        if (!t_defer.hq.empty())
            if (const int rc = host_flush(); rc != ECG_OK) return rc;
        t_defer.q.push_back(DeferredCall{this, st, B, ops, std::vector<uint8_t*>(blocks, blocks + nblocks)});
        return t_defer.q.size() >= flush_at() ? batch_flush() : ECG_OK;
    }
    return launch_direct(*ops, blocks, B, st);
}

// The context's completion-flag page (zero-copy host calls), allocated on first use.
static bool flags_ready(HostCtx& c) {
    if (c.flags) return true;
    if (hipHostMalloc((void**)&c.flags, kFlagSlots * sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess) {
        (void)hipGetLastError();
        c.flags = nullptr;
        return false;
    }
    if (hipHostGetDevicePointer((void**)&c.flags_dev, c.flags, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(c.flags);
        c.flags = nullptr;
        return false;
    }
    memset(c.flags, 0, kFlagSlots * sizeof(unsigned));
    return true;
}

// Poll flags[0, n) until each holds seq (spinning for the first 200 us, then yielding the core between
// polls).  A flag that does not arrive within 100 ms hands over to the
// stream (a fault is reported there; a slow launch just finishes).  Every 64 flagged calls the stream is
// queried so that the runtime retires the completed launches it never waited for.
static int wait_flags(HostCtx& c, int n, unsigned seq, hipStream_t st) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) {
        while (__atomic_load_n(&c.flags[i], __ATOMIC_ACQUIRE) != seq) {
            const auto waited = std::chrono::steady_clock::now() - t0;
            if (waited < std::chrono::microseconds(200))
                __builtin_ia32_pause();
            else
                std::this_thread::yield();  // queued behind other work: stop burning the core
            if (waited > std::chrono::milliseconds(100)) {
                ECG_HIP(hipStreamSynchronize(st));
                for (int j = i; j < n; j++)
                    if (__atomic_load_n(&c.flags[j], __ATOMIC_ACQUIRE) != seq) {
                        set_last_error("zero-copy call: a completion flag never arrived");
                        return ECG_EHIP;
                    }
                c.unreaped = 0;
                return ECG_OK;
            }
        }
    }
    if (++c.unreaped >= 64) {
        c.unreaped = 0;
        const hipError_t e = hipStreamQuery(st);
        if (e != hipSuccess && e != hipErrorNotReady) {
            set_last_error(std::string("hipStreamQuery: ") + hipGetErrorString(e));
            return ECG_EHIP;
        }
    }
    return ECG_OK;
}

namespace {

// Resident call worker of a device (ECG_OPT_CALL_WORKER > 0; gf_kernels.hpp WorkerArgs).
// A small synchronous host-tier call normally pays a kernel launch (~4 us of an ~11 us RS(6,4) 1 KiB call);
// with the worker, a resident kernel polls a descriptor ring in pinned host memory and the call only
// writes its descriptor (profiles/r03/persist/persist_probe.hip: 11.4 -> 4.9 us).  One call at a time goes through it
// (try_lock): concurrent callers take the launch path, so concurrency is never serialised behind it.
// The worker runs on a HIGH-PRIORITY stream: HIP maps streams onto a few hardware queues, and a kernel
// that stays resident on a queue shared with another stream holds that stream's work behind it until it
// exits (measured: 28 ms for one of 8 normal streams, none with the worker on a high-priority stream;
// profiles/r03/persist/queue_interference.log).  A process that issues its own work on high-priority
// streams shares that queue -- hence the option is off by default.  The worker exits by itself after the
// option's idle time without a call, takes no call after 50 ms (the waiting call then starts the next
// generation, so the queue is released at least that often), and stops at process exit.
struct CallWorker {
    static constexpr double kLifeMs = 50.0;
    std::mutex mu;
    bool ready = false, broken = false, running = false;
    int device = 0;
    hipStream_t st = nullptr;
    uint8_t* host = nullptr;  // pinned, mapped: ring [0, 1024), flags [1024, 1280), stop @2048, exit_info @2112
    uint8_t* host_dev = nullptr;
    uint8_t* dmem = nullptr;  // device: mailbox [0, 1024), mailbox seqs + exit word @1024
    unsigned seq = 0, gen = 0;
    int W = 0;
    unsigned long long ticks_per_us = 100;
    long long idle_us = 0, gen_idle_us = 0;  // the option now / the running generation's idle limit
    long long calls = 0, launches = 0, relaunches = 0;
    // A call that does not complete within 100 ms (queued behind a long kernel, e.g.) turns the worker off
    // for a cooldown that doubles per consecutive timeout (1 s .. 64 s); calls take the launch path meanwhile.
    // `broken` stays for what cannot recover: initialisation failed.
    std::chrono::steady_clock::time_point off_until{};
    int timeouts_in_row = 0;
    long long timeouts = 0;
    bool cooling() const { return std::chrono::steady_clock::now() < off_until; }
    void back_off() {
        timeouts++;
        const int sh = std::min(timeouts_in_row++, 6);
        off_until = std::chrono::steady_clock::now() + std::chrono::seconds(1LL << sh);
    }

    WorkerDesc* ring() { return (WorkerDesc*)host; }
    unsigned* flags() { return (unsigned*)(host + 1024); }
    volatile unsigned* stopw() { return (volatile unsigned*)(host + 2048); }
    unsigned* exit_info() { return (unsigned*)(host + 2112); }

    bool init(int dev) {
        device = dev;
        int lo = 0, hi = 0, khz = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return false;
        if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, hi) != hipSuccess) return false;
        if (hipHostMalloc((void**)&host, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return false;
        if (hipHostGetDevicePointer((void**)&host_dev, host, 0) != hipSuccess) return false;
        memset(host, 0, 4096);
        if (hipMalloc((void**)&dmem, 2048) != hipSuccess) return false;
        if (hipMemsetAsync(dmem, 0, 2048, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return false;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) return false;
        ticks_per_us = (unsigned long long)khz / 1000ULL;
        if (ticks_per_us == 0) ticks_per_us = 1;
        ready = true;
        return true;
    }
    // every workgroup of the current generation has exited (it writes `gen` as it leaves)
    bool gone() {
        if (!running) return true;
        for (int w = 0; w < W; w++)
            if (__atomic_load_n(&exit_info()[w], __ATOMIC_ACQUIRE) != gen) return false;
        running = false;
        return true;
    }
    // Start a generation at call `start` (only while none is running).  The call's flags are cleared first:
    // a generation that left (or was stopped) may have posted some of them for this very call, and the new
    // one redoes the call from the start.  Flags left over from it would let the host finish the call
    // while a workgroup of the new generation still rewrites the call's outputs -- into staging memory
    // the host hands to the next call (seen as a wrong decode in the 8-thread x 2000 soak, where call
    // sizes change and generations are restarted often).
    int launch(int workgroups, unsigned start) {
        unsigned* f = flags() + (start % kWorkerSlots) * kWorkerMaxWG;
        for (int w = 0; w < kWorkerMaxWG; w++) __atomic_store_n(&f[w], 0u, __ATOMIC_RELAXED);
        WorkerArgs a;
        memset(&a, 0, sizeof a);
        if (++gen == 0) ++gen;
        a.ring = (const WorkerDesc*)host_dev;
        a.flags = (unsigned*)(host_dev + 1024);
        a.stop = (const unsigned*)(host_dev + 2048);
        a.mbox = (WorkerDesc*)dmem;
        a.mbseq = (unsigned*)(dmem + 1024);
        a.exit_info = (unsigned*)(host_dev + 2112);
        a.start_seq = start;
        a.gen = gen;
        a.max_polls = 1u << 24;
        a.idle_ticks = (unsigned long long)idle_us * ticks_per_us;
        a.life_ticks = (unsigned long long)(kLifeMs * 1000.0) * ticks_per_us;
        *stopw() = 0;
        const hipError_t e = launch_call_worker(a, workgroups, st);
        if (e != hipSuccess) {
            set_last_error(std::string("call worker launch: ") + hipGetErrorString(e));
            return ECG_EHIP;
        }
        W = workgroups;
        gen_idle_us = idle_us;
        running = true;
        launches++;
        return ECG_OK;
    }
    // stop the running generation and wait until it is gone (bounded: it exits at its next poll)
    int stop() {
        if (!running) return ECG_OK;
        *stopw() = 1;
        const auto t0 = std::chrono::steady_clock::now();
        while (!gone()) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                if (hipStreamSynchronize(st) != hipSuccess) return ECG_EHIP;
                running = false;
                break;
            }
            __builtin_ia32_pause();
        }
        *stopw() = 0;
        return ECG_OK;
    }
    bool done(unsigned slot, unsigned s) {
        const unsigned* f = flags() + slot * kWorkerMaxWG;
        for (int w = 0; w < W; w++)
            if (__atomic_load_n(&f[w], __ATOMIC_ACQUIRE) != s) return false;
        return true;
    }
    // One call: 0 = done, 1 = not taken (use the launch path), < 0 = error.
    int call(int dev_id, const ProgramSet& ps, const LinearOp& op, uint8_t* const* dev, long long B) {
        if (broken || cooling()) return 1;
        if (!ready && !init(dev_id)) {
            broken = true;
            return 1;
        }
        idle_us = get_option(ECG_OPT_CALL_WORKER);
        const int need = (int)std::max(1LL, ((B >> 2) + kLatThreads - 1) / kLatThreads);
        if (need > kWorkerMaxWG) return 1;
        unsigned s = ++seq;
        if (s == 0) s = ++seq;
        const unsigned slot = s % kWorkerSlots;
        // payload, then the four sequence numbers (x86 stores become visible in program order)
        WorkerDesc& d = ring()[slot];
        unsigned pay[60] = {};
        pay[WF_K] = (unsigned)op.k_in();
        pay[WF_M] = (unsigned)op.m_out();
        pay[WF_B] = (unsigned)B;
        pay[WF_BINARY] = ps.binary ? 1u : 0u;
        auto put64 = [&](int q, const void* p) {
            pay[q] = (unsigned)(uintptr_t)p;
            pay[q + 1] = (unsigned)((uintptr_t)p >> 32);
        };
        put64(WF_TABS, ps.d_tabs);
        for (int j = 0; j < op.k_in(); j++) put64(WF_IN + 2 * j, dev[op.src_ids[j]]);
        for (int p = 0; p < op.m_out(); p++) put64(WF_OUT + 2 * p, dev[op.dst_ids[p]]);
        for (int q = 0; q < 60; q++) d.w[worker_pos(q)] = pay[q];
        std::atomic_thread_fence(std::memory_order_release);
        for (int l = 0; l < 4; l++) __atomic_store_n(&d.w[16 * l], s, __ATOMIC_RELEASE);
        // a generation too narrow for this call, or started under another idle limit, makes way for a new one
        if (!gone() && (W < need || gen_idle_us != idle_us) && stop() != ECG_OK) return ECG_EHIP;
        if (!running && launch(std::max(need, 1), s) != ECG_OK) {
            back_off();
            return 1;
        }
        const auto t0 = std::chrono::steady_clock::now();
        auto next_check = t0 + std::chrono::microseconds(20);
        while (!done(slot, s)) {
            const auto t = std::chrono::steady_clock::now();
            if (t > next_check) {
                next_check = t + std::chrono::microseconds(20);
                if (gone() && !done(slot, s)) {  // the generation left before taking the call: a new one takes it
                    relaunches++;
                    if (launch(std::max(need, W), s) != ECG_OK) {
                        back_off();
                        return 1;
                    }
                }
            }
            if (t - t0 > std::chrono::milliseconds(100)) {
                // the generation is gone once stopped and its stream drained; a call it did not finish takes
                // the launch path (its outcome is that path's status, so no error is recorded here)
                (void)stop();
                (void)hipStreamSynchronize(st);
                back_off();
                if (!done(slot, s)) return 1;
                calls++;
                return 0;
            }
            if (t - t0 > std::chrono::microseconds(200)) std::this_thread::yield();
            else __builtin_ia32_pause();
        }
        calls++;
        timeouts_in_row = 0;
        return 0;
    }
};

CallWorker g_worker[kMaxDevices];

// At process exit: tell running workers to stop (a store to pinned host memory) and wait briefly for them
// to leave -- no HIP call, the runtime may already be going down.  They would leave by themselves within
// their idle time anyway.
struct WorkerReaper {
    ~WorkerReaper() {
        for (CallWorker& w : g_worker) {
            // a thread still inside a call (detached threads run on during exit) keeps its worker: that
            // generation leaves by itself within its idle time
            std::unique_lock<std::mutex> lk(w.mu, std::try_to_lock);
            if (!lk.owns_lock() || !w.ready || !w.running) continue;
            *w.stopw() = 1;
            const auto t0 = std::chrono::steady_clock::now();
            while (!w.gone() && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20)) __builtin_ia32_pause();
        }
    }
} g_worker_reaper;

}  // namespace

int call_worker_stats(long long* calls, long long* launches, long long* relaunches, int* disabled) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDevices) return ECG_EINVAL;
    CallWorker& w = g_worker[dev];
    std::lock_guard<std::mutex> lk(w.mu);
    if (calls) *calls = w.calls;
    if (launches) *launches = w.launches;
    if (relaunches) *relaunches = w.relaunches;
    if (disabled) *disabled = (w.broken || w.cooling()) ? 1 : 0;
    return ECG_OK;
}

// Host-buffer tier (the reference's per-stripe calls on host memory).  Device slots are assigned to the
// blocks that must be uploaded first (read before any op writes them), then to the rest, so the
// inputs form one contiguous range.  Small calls (the proxy's 1 KiB - 64 KiB blocks) gather those
// inputs into the leased context's pinned staging area with memcpy and move them with ONE H2D copy, and bring
// every written block back with ONE D2H copy: two DMA transfers per call instead of one pageable copy
// per block (each pageable copy is a driver-staged round trip).  Large calls copy block by block.
int Engine::run_host(const std::vector<LinearOp>& ops, uint8_t* const* blocks, int nblocks, long long B) {
    if (B < 0) return ECG_EINVAL;
    if (t_defer.active && t_defer.host_defer && !ops.empty() && B > 0) {
        const int rc = record_host(this, ops, blocks, nblocks, B);
        if (rc <= 0) return rc;  // recorded (or refused); 1 = not deferrable: run it now, below
    }
    if (const int rc = batch_flush_pending(); rc != ECG_OK) return rc;  // keep call order with recorded calls
    if (ops.empty() || B == 0) return ECG_OK;
    CtxLease lease(device_);
    HostCtx& c = *lease;
    if (!c.stream) ECG_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    hipStream_t st = c.stream;
    // per-call bookkeeping in per-thread buffers (a 1 KiB call costs ~10 us of which the host's share is
    // what allocation would add to)
    thread_local std::vector<char> upload, written, used, produced;
    thread_local std::vector<int> slot;
    thread_local std::vector<uint8_t*> dev;
    upload.assign(nblocks, 0);
    written.assign(nblocks, 0);
    used.assign(nblocks, 0);
    {
        produced.assign(nblocks, 0);
        for (const LinearOp& op : ops) {
            for (int id : op.src_ids) {
                if (id < 0 || id >= nblocks || !blocks[id]) return ECG_EINVAL;
                if (!produced[id]) upload[id] = 1;
                used[id] = 1;
            }
            for (int id : op.dst_ids) {
                if (id < 0 || id >= nblocks || !blocks[id]) return ECG_EINVAL;
                produced[id] = written[id] = used[id] = 1;
            }
        }
    }
    slot.assign(nblocks, -1);
    int nslots = 0, n_up = 0;
    for (int id = 0; id < nblocks; id++)
        if (upload[id]) slot[id] = nslots++;
    n_up = nslots;
    for (int id = 0; id < nblocks; id++)
        if (used[id] && slot[id] < 0) slot[id] = nslots++;
    const size_t pitch = ((size_t)B + 255) & ~(size_t)255;
    if (c.cap < pitch * nslots) {
        ECG_HIP(hipStreamSynchronize(st));
        if (c.scratch) (void)hipFree(c.scratch);
        c.scratch = nullptr;
        c.cap = 0;
        ECG_HIP(hipMalloc(&c.scratch, pitch * nslots));
        c.cap = pitch * nslots;
    }
    dev.assign(nblocks, nullptr);
    for (int id = 0; id < nblocks; id++)
        if (slot[id] >= 0) dev[id] = c.scratch + (size_t)slot[id] * pitch;
    const bool staged = (size_t)B <= kStagedMaxBlock && pitch * nslots <= kStagedMaxBytes;
    if (staged && c.pinned_cap < pitch * nslots) {
        ECG_HIP(hipStreamSynchronize(st));
        if (c.pinned) (void)hipHostFree(c.pinned);
        c.pinned = nullptr;
        c.pinned_cap = 0;
        const size_t cap = std::max(pitch * nslots, (size_t)1 << 20);
        ECG_HIP(hipHostMalloc((void**)&c.pinned, cap, hipHostMallocMapped | hipHostMallocCoherent));
        ECG_HIP(hipHostGetDevicePointer((void**)&c.pinned_dev, c.pinned, 0));
        c.pinned_cap = cap;
    }
    // zero-copy: the kernel streams the (tiny) blocks straight over PCIe from / to the mapped staging area
    const long long zc_max = get_option(ECG_OPT_ZEROCOPY_BYTES);
    if (staged && zc_max > 0 && (long long)(pitch * nslots) <= zc_max) {
        for (int id = 0; id < nblocks; id++) {
            if (slot[id] < 0) continue;
            dev[id] = c.pinned_dev + (size_t)slot[id] * pitch;
            if (upload[id]) memcpy(c.pinned + (size_t)slot[id] * pitch, blocks[id], (size_t)B);
        }
        // Completion by flags: every workgroup posts a flag once its stores are visible to the host, and the
        // host polls the flags instead of synchronizing the stream -- the runtime's completion round trip is
        // ~4 us of a ~14 us call (profiles/r02/small_call/small_call.cpp).  Only for launches whose
        // vector path covers every byte and that fit the flag page; anything else synchronizes as before.
        // the resident call worker, when enabled: one op of at most 16 inputs and 4 outputs, blocks of at
        // most 16 KiB in 4-byte lanes, tables already resident; anything else takes the launch path below
        if (ops.size() == 1 && B > 0 && (B % 4) == 0 && get_option(ECG_OPT_CALL_WORKER) > 0) {
            const LinearOp& op = ops[0];
            if (op.k_in() >= 1 && op.k_in() <= kWorkerMaxSrc && op.m_out() >= 1 && op.m_out() <= kWorkerMaxRows) {
                CallWorker& wk = g_worker[device_];
                std::unique_lock<std::mutex> lk(wk.mu, std::try_to_lock);
                if (lk.owns_lock()) {
                    int status = ECG_OK;
                    std::shared_ptr<ProgramSet> ps = program_set(&op, 1, &status, st);
                    if (!ps) return status;
                    if (ps->ready.load(std::memory_order_acquire) || hipEventQuery(ps->ready_ev) == hipSuccess) {
                        (void)ps->ensure_ready(st);  // marks the set ready (its upload has completed)
                        const int rc = wk.call(device_, *ps, op, dev.data(), B);
                        if (rc < 0) return rc;
                        if (rc == 0) {
                            for (int id = 0; id < nblocks; id++)
                                if (written[id]) memcpy(blocks[id], c.pinned + (size_t)slot[id] * pitch, (size_t)B);
                            return lease.done();
                        }
                    }
                }
            }
        }
        bool flagged = (B % 16) == 0 && flags_ready(c);
        for (const LinearOp& op : ops)
            flagged &= op.k_in() > 0 && op.k_in() <= kInlineSrc && op.m_out() <= kInlineDst;
        const unsigned seq = ++c.seq == 0 ? ++c.seq : c.seq;  // flags start at 0: never post 0
        int nflags = 0;
        for (const LinearOp& op : ops) {
            // >= workgroups x row tiles of either latency kernel (4 bytes per lane is the finer grid)
            const long long wg_max = ((B / 4 + kLatThreads - 1) / kLatThreads) * op.m_out();
            const bool f = flagged && nflags + wg_max <= kFlagSlots;
            flagged = f;
            int posted = 0;
            int rc = launch_one(op, dev.data(), B, st, /*host_tier=*/true, /*latency=*/true,
                                f ? c.flags_dev + nflags : nullptr, seq, &posted);
            if (rc != ECG_OK) {
                (void)hipStreamSynchronize(st);
                return rc;
            }
            nflags += posted;
        }
        if (flagged) {
            if (const int rc = wait_flags(c, nflags, seq, st); rc != ECG_OK) return rc;
        } else {
            ECG_HIP(hipStreamSynchronize(st));
        }
        for (int id = 0; id < nblocks; id++)
            if (written[id]) memcpy(blocks[id], c.pinned + (size_t)slot[id] * pitch, (size_t)B);
        return lease.done();
    }
    if (staged) {
        for (int id = 0; id < nblocks; id++)
            if (upload[id]) memcpy(c.pinned + (size_t)slot[id] * pitch, blocks[id], (size_t)B);
        if (n_up > 0) ECG_HIP(hipMemcpyAsync(c.scratch, c.pinned, pitch * n_up, hipMemcpyHostToDevice, st));
    }
    // large blocks: pageable copies, one per run of blocks that are contiguous both in host memory and in
    // the device scratch (the proxy's k slices of one value buffer, proxy.cpp:337-339, move as ONE copy:
    // a single large pageable copy runs at the pinned rate, per-block 1 MiB copies at half of it).
    // The caller's pages are deliberately NOT registered (hipHostRegister) for the call: the runtime
    // then treats every copy that touches those pages as pinned -- including other threads' copies of
    // neighbouring heap objects -- and unregistering under such a copy faulted the GPU
    // (tests/test_gpu_stress.py).
    if (!staged) {
        int id = 0;
        while (id < nblocks) {
            if (!upload[id]) {
                id++;
                continue;
            }
            int j = id + 1;
            while (j < nblocks && upload[j] && blocks[j] == blocks[j - 1] + B && dev[j] == dev[j - 1] + B) j++;
            ECG_HIP(hipMemcpyAsync(dev[id], blocks[id], (size_t)B * (j - id), hipMemcpyHostToDevice, st));
            id = j;
        }
    }
    for (const LinearOp& op : ops) {
        int rc = launch_one(op, dev.data(), B, st, /*host_tier=*/true);
        if (rc != ECG_OK) {
            (void)hipStreamSynchronize(st);
            return rc;
        }
    }
    if (staged) {
        int lo = nslots, hi = -1;
        for (int id = 0; id < nblocks; id++)
            if (written[id]) {
                lo = std::min(lo, slot[id]);
                hi = std::max(hi, slot[id]);
            }
        if (hi >= lo) {
            ECG_HIP(hipMemcpyAsync(c.pinned + (size_t)lo * pitch, c.scratch + (size_t)lo * pitch,
                                   (size_t)(hi - lo) * pitch + (size_t)B, hipMemcpyDeviceToHost, st));
            ECG_HIP(hipStreamSynchronize(st));
            for (int id = 0; id < nblocks; id++)
                if (written[id]) memcpy(blocks[id], c.pinned + (size_t)slot[id] * pitch, (size_t)B);
        } else {
            ECG_HIP(hipStreamSynchronize(st));
        }
        return lease.done();
    }
    int id = 0;
    while (id < nblocks) {
        if (!written[id]) {
            id++;
            continue;
        }
        int j = id + 1;
        while (j < nblocks && written[j] && blocks[j] == blocks[j - 1] + B && dev[j] == dev[j - 1] + B) j++;
        ECG_HIP(hipMemcpyAsync(blocks[id], dev[id], (size_t)B * (j - id), hipMemcpyDeviceToHost, st));
        id = j;
    }
    ECG_HIP(hipStreamSynchronize(st));
    return lease.done();
}

// Row split of a batched launch (ECG_OPT_ROW_SPLIT, include/ecg.h): when every program's output rows read
// disjoint input sets of one size, each (stripe, row) runs as its own launch stripe over that row's inputs
// only.  A PC merge's 40 -> 5 XOR then streams 8 blocks per workgroup instead of 40 (the fused form ran
// at 0.72 of HBM peak against 0.76 for rows, profiles/r03/final/workloads/bench_pc-merge.log).  Rows
// then run in different workgroups, so no output block may be an input block of the same stripe: the
// split is taken only when the outputs provably overlap no input (disjoint spans, or, for equal stripe
// strides, no output within B bytes of an input of its stripe).  Returns R = rows per program (0 = no
// split) and the split programs, program p * R + r = row r of program p.
static int row_split(const std::vector<LinearOp>& progs, int S, const void* in_base, long long iss, long long ibs,
                     const void* out_base, long long oss, long long obs, long long B, bool has_stripe_of,
                     std::vector<LinearOp>& rows) {
    const long long min_k = get_option(ECG_OPT_ROW_SPLIT);
    const int k = progs[0].k_in(), m = progs[0].m_out();
    if (min_k <= 0 || k < min_k || m < 2 || k % m || (long long)S * m > 0x7fffffffLL) return 0;
    // the disjointness tests below bound spans by their last block, which needs non-negative strides
    if (iss < 0 || ibs < 0 || oss < 0 || obs < 0) return 0;
    const int kr = k / m;
    int max_src = 0, max_dst = 0;
    for (const LinearOp& op : progs) {
        if (op.k_in() != k || op.m_out() != m || op.coef.size() != (size_t)k * m) return 0;
        for (int j = 0; j < k; j++) {
            int users = 0;
            for (int r = 0; r < m; r++) users += op.coef[(size_t)r * k + j] != 0;
            if (users != 1) return 0;
        }
        for (int r = 0; r < m; r++) {
            int n = 0;
            for (int j = 0; j < k; j++) n += op.coef[(size_t)r * k + j] != 0;
            if (n != kr) return 0;
        }
        for (int id : op.src_ids) max_src = std::max(max_src, id);
        for (int id : op.dst_ids) max_dst = std::max(max_dst, id);
    }
    const uintptr_t ib = (uintptr_t)in_base, ob = (uintptr_t)out_base;
    bool safe = false;
    if (!has_stripe_of) {
        const uintptr_t i1 = ib + (uintptr_t)((S - 1) * iss + max_src * ibs + B);
        const uintptr_t o1 = ob + (uintptr_t)((S - 1) * oss + max_dst * obs + B);
        safe = i1 <= ob || o1 <= ib;
    }
    if (!safe && iss == oss) {
        safe = true;
        for (const LinearOp& op : progs)
            for (int d : op.dst_ids)
                for (int j : op.src_ids) {
                    const long long delta = (long long)(ob + (uintptr_t)(d * obs)) - (long long)(ib + (uintptr_t)(j * ibs));
                    if (delta > -B && delta < B) safe = false;
                }
    }
    if (!safe) return 0;
    rows.clear();
    for (const LinearOp& op : progs)
        for (int r = 0; r < m; r++) {
            LinearOp one;
            one.dst_ids.push_back(op.dst_ids[r]);
            for (int j = 0; j < k; j++)
                if (const uint8_t c = op.coef[(size_t)r * k + j]) {
                    one.src_ids.push_back(op.src_ids[j]);
                    one.coef.push_back(c);
                }
            rows.push_back(std::move(one));
        }
    return m;
}

int Engine::run_strided(const std::vector<LinearOp>& progs, const int* d_prog_of_stripe, int S,
                        const void* in_base, long long in_sstride, long long in_bstride, void* out_base,
                        long long out_sstride, long long out_bstride, long long B, hipStream_t st,
                        const int* d_stripe_of) {
    if (S < 0 || B < 0) return ECG_EINVAL;
    if (S == 0 || B == 0) return ECG_OK;  // empty batch: nothing to read or write
    if (!in_base || !out_base) return ECG_EINVAL;
    if (const int rc = batch_flush_pending(); rc != ECG_OK) return rc;
    if (progs.size() > 1 && !d_prog_of_stripe) return ECG_EINVAL;
    thread_local std::vector<LinearOp> rows;
    const int R = row_split(progs, S, in_base, in_sstride, in_bstride, out_base, out_sstride, out_bstride, B,
                            d_stripe_of != nullptr, rows);
    int status = ECG_OK;
    std::shared_ptr<ProgramSet> ps = R ? program_set(rows, &status, st) : program_set(progs, &status, st);
    if (!ps) return status;
    if (const int rc = ps->ensure_ready(st); rc != ECG_OK) return rc;
    GfLaunch a;
    memset(&a, 0, sizeof(a));
    a.tabs = ps->d_tabs;
    a.src_ids = ps->d_src;
    a.dst_ids = ps->d_dst;
    a.prog_of_stripe = progs.size() > 1 ? d_prog_of_stripe : nullptr;
    a.stripe_of = d_stripe_of;
    a.in_base = (const uint8_t*)in_base;
    a.out_base = (uint8_t*)out_base;
    a.in_sstride = in_sstride;
    a.in_bstride = in_bstride;
    a.out_sstride = out_sstride;
    a.out_bstride = out_bstride;
    a.B = B;
    a.k = ps->k;
    a.m = ps->m;
    a.S = R ? S * R : S;
    a.row_split = R;
    a.MT = ps->MT;
    a.rtiles = ps->rtiles;
    a.binary = ps->binary ? 1 : 0;
    const bool vec_ok = aligned16(in_base) && aligned16(out_base) && (in_sstride % 16 == 0) &&
                        (in_bstride % 16 == 0) && (out_sstride % 16 == 0) && (out_bstride % 16 == 0);
    ECG_HIP(launch_gf(a, GF_MODE_STRIDED, vec_ok, st));
    note_launch(*ps, st);
    return ECG_OK;
}

int Engine::run_ptrs(const LinearOp& prog, const uint8_t* const* d_src, uint8_t* const* d_dst, int S, long long B,
                     bool aligned, hipStream_t st, bool apart) {
    if (S < 0 || B < 0) return ECG_EINVAL;
    if (S == 0 || B == 0) return ECG_OK;
    if (!d_src || !d_dst) return ECG_EINVAL;
    int status = ECG_OK;
    std::shared_ptr<ProgramSet> ps = program_set(&prog, 1, &status, st);
    if (!ps) return status;
    if (const int rc = ps->ensure_ready(st); rc != ECG_OK) return rc;
    GfLaunch a;
    memset(&a, 0, sizeof(a));
    a.tabs = ps->d_tabs;
    a.src_ids = ps->d_src;
    a.dst_ids = ps->d_dst;
    a.src_ptrs = d_src;
    a.dst_ptrs = d_dst;
    a.B = B;
    a.k = ps->k;
    a.m = ps->m;
    a.S = S;
    a.MT = ps->MT;
    a.rtiles = ps->rtiles;
    a.binary = ps->binary ? 1 : 0;
    a.grid_map = apart ? 2 : 0;  // the auto map's layout hint (gf_kernels.hip outputs_in_stripe)
    ECG_HIP(launch_gf(a, GF_MODE_PTRS, aligned, st));
    note_launch(*ps, st);
    return ECG_OK;
}

// Page-locked (hipHostMalloc'd or registered) host memory, as opposed to ordinary pageable memory.
static bool host_pinned(const void* p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

int Engine::run_host_pipeline(const LinearOp& prog, const void* h_in, long long in_sstride, long long in_bstride,
                              void* h_out, long long out_sstride, long long out_bstride, long long B, int S,
                              int chunk) {
    if (S < 0 || B < 0 || prog.k_in() < 1 || prog.m_out() < 1) return ECG_EINVAL;
    if (S == 0 || B == 0) return ECG_OK;
    if (!h_in || !h_out) return ECG_EINVAL;
    if (const int rc = batch_flush_pending(); rc != ECG_OK) return rc;
    if (chunk < 1) chunk = 16;
    if (chunk > S) chunk = S;
    const int kin = prog.k_in(), mout = prog.m_out();
    const size_t pitch = ((size_t)B + 255) & ~(size_t)255;
    const size_t slot_in = (size_t)chunk * kin * pitch, slot_out = (size_t)chunk * mout * pitch;
    CtxLease lease(device_);
    HostCtx& c = *lease;
    if (!c.pipe_ready) {
        for (int i = 0; i < 3; i++) {
            ECG_HIP(hipStreamCreateWithFlags(&c.pstream[i], hipStreamNonBlocking));
            ECG_HIP(hipEventCreateWithFlags(&c.in_done[i], hipEventDisableTiming));
            ECG_HIP(hipEventCreateWithFlags(&c.comp_done[i], hipEventDisableTiming));
            ECG_HIP(hipEventCreateWithFlags(&c.out_done[i], hipEventDisableTiming));
        }
        c.pipe_ready = true;
    }
    if (c.pslot_cap < 3 * (slot_in + slot_out)) {
        for (int i = 0; i < 3; i++) ECG_HIP(hipStreamSynchronize(c.pstream[i]));
        if (c.pslot) (void)hipFree(c.pslot);
        c.pslot = nullptr;
        c.pslot_cap = 0;
        ECG_HIP(hipMalloc(&c.pslot, 3 * (slot_in + slot_out)));
        c.pslot_cap = 3 * (slot_in + slot_out);
    }
    // the device program reads compact slot blocks 0..kin-1 and writes 0..mout-1
    LinearOp dev = prog;
    for (int j = 0; j < kin; j++) dev.src_ids[j] = j;
    for (int p = 0; p < mout; p++) dev.dst_ids[p] = p;
    int status = ECG_OK;
    hipStream_t s_in = c.pstream[0], s_comp = c.pstream[1], s_out = c.pstream[2];
    std::shared_ptr<ProgramSet> ps = program_set(&dev, 1, &status, s_comp);
    if (!ps) return status;
    if (const int rc = ps->ensure_ready(s_comp); rc != ECG_OK) return rc;
    const uint8_t* hin = (const uint8_t*)h_in;
    uint8_t* hout = (uint8_t*)h_out;
    const bool in_pinned = host_pinned(h_in), out_pinned = host_pinned(h_out);
    const int nchunks = (int)((S + (long long)chunk - 1) / chunk);
    auto issue_out = [&](int it) -> int {  // D2H of chunk it, behind its kernel
        const int s0 = it * chunk, n = std::min(chunk, S - s0), slot = it % 3;
        uint8_t* dout = c.pslot + (size_t)slot * (slot_in + slot_out) + slot_in;
        ECG_HIP(hipStreamWaitEvent(s_out, c.comp_done[slot], 0));
        for (int p = 0; p < mout; p++)
            ECG_HIP(hipMemcpy2DAsync(hout + (size_t)s0 * out_sstride + (size_t)prog.dst_ids[p] * out_bstride,
                                     (size_t)out_sstride, dout + (size_t)p * pitch, (size_t)mout * pitch, (size_t)B,
                                     (size_t)n, hipMemcpyDeviceToHost, s_out));
        ECG_HIP(hipEventRecord(c.out_done[slot], s_out));
        return ECG_OK;
    };
    // A copy to or from pageable memory (the proxy's own vectors) returns only once the runtime has moved
    // the bytes, so issued from one thread the input and output copies of a pageable batch run one after
    // the other: RS(10,4) 1 MiB encode 36 GiB/s of data, the H2D and D2H times added.  PCIe is full
    // duplex: with either side pageable, a second host thread issues the output copies (50 GiB/s, the
    // pinned rate; profiles/r02/pipeline/).  Copying pageable runs of consecutive blocks as 1-D copies,
    // which the runtime pins per copy above 1 MiB, measured slower than these 2-D copies and was dropped.
    // Chunk it's copies wait (host side) for its kernel to be enqueued; the kernel that reuses a slot waits
    // until the copies that drain it are enqueued, so every event wait refers to the intended record.
    struct OutThread {
        std::mutex mu;
        std::condition_variable cv;
        int comp_issued = 0, out_issued = 0, rc = ECG_OK;
        std::string msg;  // the copy thread's error message (last_error is per thread)
        bool stop = false;
        std::thread th;
        void finish() {
            if (!th.joinable()) return;
            {
                std::lock_guard<std::mutex> lk(mu);
                stop = true;
            }
            cv.notify_all();
            th.join();
        }
        ~OutThread() { finish(); }
    } ot;
    const bool split = !in_pinned || !out_pinned;
    if (split) {
        ot.th = std::thread([&] {
            if (hipSetDevice(device_) != hipSuccess) {  // the current device is per host thread
                std::lock_guard<std::mutex> lk(ot.mu);
                ot.rc = ECG_EHIP;
                ot.msg = "host pipeline: hipSetDevice failed on the copy thread";
                ot.cv.notify_all();
                return;
            }
            for (int it = 0; it < nchunks; it++) {
                {
                    std::unique_lock<std::mutex> lk(ot.mu);
                    ot.cv.wait(lk, [&] { return ot.comp_issued > it || ot.stop; });
                    if (ot.comp_issued <= it) return;  // stopped early (error on the issuing thread)
                }
                const int rc = issue_out(it);
                {
                    std::lock_guard<std::mutex> lk(ot.mu);
                    if (rc != ECG_OK) {
                        ot.rc = rc;
                        ot.msg = last_error_string();
                    } else {
                        ot.out_issued = it + 1;
                    }
                }
                ot.cv.notify_all();
                if (rc != ECG_OK) return;
            }
        });
    }
    for (int it = 0; it < nchunks; it++) {
        const int s0 = it * chunk, n = std::min(chunk, S - s0), slot = it % 3;
        const bool reuse = it >= 3;
        uint8_t* din = c.pslot + (size_t)slot * (slot_in + slot_out);
        uint8_t* dout = din + slot_in;
        if (reuse) ECG_HIP(hipStreamWaitEvent(s_in, c.comp_done[slot], 0));  // slot's inputs consumed
        for (int j = 0; j < kin; j++)
            ECG_HIP(hipMemcpy2DAsync(din + (size_t)j * pitch, (size_t)kin * pitch,
                                     hin + (size_t)s0 * in_sstride + (size_t)prog.src_ids[j] * in_bstride,
                                     (size_t)in_sstride, (size_t)B, (size_t)n, hipMemcpyHostToDevice, s_in));
        ECG_HIP(hipEventRecord(c.in_done[slot], s_in));
        ECG_HIP(hipStreamWaitEvent(s_comp, c.in_done[slot], 0));
        if (reuse) {
            if (split) {  // the copies draining this slot (chunk it - 3) must be enqueued first
                std::unique_lock<std::mutex> lk(ot.mu);
                ot.cv.wait(lk, [&] { return ot.out_issued >= it - 2 || ot.rc != ECG_OK; });
                if (ot.rc != ECG_OK) {
                    set_last_error(ot.msg);
                    return ot.rc;
                }
            }
            ECG_HIP(hipStreamWaitEvent(s_comp, c.out_done[slot], 0));  // slot's outputs copied out
        }
        GfLaunch a;
        memset(&a, 0, sizeof(a));
        a.tabs = ps->d_tabs;
        a.src_ids = ps->d_src;
        a.dst_ids = ps->d_dst;
        a.in_base = din;
        a.out_base = dout;
        a.in_sstride = (long long)(kin * pitch);
        a.in_bstride = (long long)pitch;
        a.out_sstride = (long long)(mout * pitch);
        a.out_bstride = (long long)pitch;
        a.B = B;
        a.k = ps->k;
        a.m = ps->m;
        a.S = n;
        a.MT = ps->MT;
        a.rtiles = ps->rtiles;
        a.binary = ps->binary ? 1 : 0;
        ECG_HIP(launch_gf(a, GF_MODE_STRIDED, true, s_comp));
        ECG_HIP(hipEventRecord(c.comp_done[slot], s_comp));
        if (split) {
            {
                std::lock_guard<std::mutex> lk(ot.mu);
                ot.comp_issued = it + 1;
            }
            ot.cv.notify_all();
        } else if (const int rc = issue_out(it); rc != ECG_OK) {
            return rc;
        }
    }
    if (split) {
        ot.th.join();
        if (ot.rc != ECG_OK) {
            set_last_error(ot.msg);
            return ot.rc;
        }
    }
    ECG_HIP(hipStreamSynchronize(s_out));
    return lease.done();
}

}  // namespace ecg
