// CPU stand-in for the HIP runtime under ThreadSanitizer (TEST INFRASTRUCTURE, never shipped).
//
// libecg's host translation units (engine, capi, codes, planning, matrix) and the host side of
// gf_kernels.hip are linked against this file instead of libamdhip64, so the engine's concurrency -- program
// cache, retirement and covers, batch scopes, deferred host calls, context pools -- runs on the CPU under
// -fsanitize=thread (tools/tsan_host.sh, tests/test_sanitize.py).  The runtime is modelled as:
//   * device memory = host memory (hipMalloc / hipHostMalloc -> aligned_alloc; a device view of pinned memory
//     is the host pointer), tracked so hipPointerGetAttributes can tell pinned from pageable;
//   * every stream operation takes effect when it is enqueued, on the calling thread -- copies, memsets and
//     kernels (below) -- so data is always ready no later than the real runtime would have it;
//   * completion is asynchronous in TIME: each operation pushes its stream's completion a few microseconds
//     (pseudo-random) past the later of now and the stream's previous completion; events, hipStreamQuery /
//     Synchronize and hipDeviceSynchronize report against those times, so the engine's not-ready paths
//     (retirement covers, upload readiness, graveyard) run;
//   * two devices: streams, events and the null stream belong to the device current at creation;
//     hipStreamPerThread is one stream per thread and device; a kernel launch on another device's stream
//     and an event record on another device's stream are errors (counted as hazards), as in HIP;
//   * kernels are emulated from their registered device names (__hipRegisterFunction): gf_vec_kernel,
//     gf_byte_kernel, gf_lat_dword_kernel and fill_splitmix_kernel are ported to loops over the same
//     workgroup -> (stripe, chunk) map and argument blocks, bit-exact, including the completion flags the
//     host-tier calls poll.  The resident call worker is not emulated (ECG_OPT_CALL_WORKER stays 0).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "gf_kernels.hpp"

namespace {

using clk = std::chrono::steady_clock;
using ecg::CoefTab;
using ecg::GfLaunch;

constexpr int kDevices = 2;  // two stand-in devices: the engine's per-device state is exercised too
thread_local int t_device = 0;

struct Stream {
    clk::time_point done{};  // completion time of the last operation enqueued
    int device = 0;
};
struct Event {
    clk::time_point done{};
    bool recorded = false;
    int device = 0;
};

// Process state, constructed on first use: the kernel file's module constructor registers its kernels
// before this file's static constructors would have run.
struct State {
    std::recursive_mutex mu;  // every field below, every Stream / Event (recursive: as_stream may register
                              // the calling thread's per-thread stream while the caller holds it)
    std::map<uintptr_t, std::pair<size_t, hipMemoryType>> allocs;  // base -> (bytes, type)
    std::vector<Stream*> streams;                               // created streams (hipDeviceSynchronize)
    Stream null_stream[kDevices];
    std::unordered_map<const void*, std::string> kernels;       // host stub -> device name
    std::atomic<uint64_t> rng{0x9E3779B97F4A7C15ull};
    // coefficient-table ranges read by launches not yet complete in device time: (lo, hi, stream, done)
    struct Reader {
        uintptr_t lo, hi;
        Stream* st;
        clk::time_point done;
    };
    std::vector<Reader> readers;
    std::atomic<long> hazards{0};
    std::atomic<long> not_ready{0};  // event / stream queries answered hipErrorNotReady (asynchrony exercised)
};
State& S() {
    static State* s = [] {  // never destroyed: threads may still call in during exit
        State* st = new State();
        for (int d = 0; d < kDevices; d++) st->null_stream[d].device = d;
        return st;
    }();
    return *s;
}
#define g_mu (S().mu)
#define g_allocs (S().allocs)
#define g_streams (S().streams)
#define g_null (S().null_stream[t_device])
#define g_kernels (S().kernels)
#define g_rng (S().rng)
#define g_readers (S().readers)
Stream* per_thread_stream() {  // one per thread and device, as in HIP
    static thread_local Stream* s[kDevices] = {};
    if (!s[t_device]) {
        Stream* p = new Stream();
        p->device = t_device;
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        g_streams.push_back(p);
        s[t_device] = p;
    }
    return s[t_device];
}

Stream* as_stream(hipStream_t st) {
    if (st == nullptr) return &g_null;
    if (st == hipStreamPerThread) return per_thread_stream();
    return reinterpret_cast<Stream*>(st);
}

// HIP_STUB_NOOP=1 (tools/host_cost.sh, host-time profiling only): kernels are not emulated and every operation
// completes at once, so what a driver measures is the library's own host work.
bool noop_mode() {
    static const bool on = getenv("HIP_STUB_NOOP") && atoi(getenv("HIP_STUB_NOOP")) == 1;
    return on;
}

// pseudo-random 1-40 us of "device time" per operation
clk::duration op_cost() {
    if (noop_mode()) return clk::duration(0);
    uint64_t x = g_rng.fetch_add(0x9E3779B97F4A7C15ull, std::memory_order_relaxed);
    x = (x ^ (x >> 31)) * 0xBF58476D1CE4E5B9ull;
    return std::chrono::microseconds(1 + (x >> 40) % 40);
}

// the operation just performed on st completes at max(now, st.done) + cost; returns that time
clk::time_point enqueue(hipStream_t st) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    Stream* s = as_stream(st);
    s->done = std::max(s->done, clk::now()) + op_cost();
    return s->done;
}

// Device-time hazard check (under g_mu): an operation on stream `st` that starts at `start` and writes or
// frees [lo, hi) must not overlap a table range still being read by a launch on ANOTHER stream (same stream:
// FIFO order).  Where the engine orders streams (hipStreamWaitEvent), `start` is already past the reader.
void check_write(Stream* st, clk::time_point start, uintptr_t lo, uintptr_t hi, const char* what) {
    auto& rd = g_readers;
    const clk::time_point now = clk::now();
    rd.erase(std::remove_if(rd.begin(), rd.end(), [&](const State::Reader& r) { return r.done < now; }), rd.end());
    for (const State::Reader& r : rd)
        if (r.st != st && r.lo < hi && lo < r.hi && r.done > start) {
            S().hazards++;
            fprintf(stderr, "hip_stub: DEVICE-TIME HAZARD: %s of [%#lx, %#lx) starts %.1f us before a launch on another "
                    "stream that reads tables there completes\n", what, (unsigned long)lo, (unsigned long)hi,
                    std::chrono::duration<double, std::micro>(r.done - start).count());
            return;
        }
}

// the start time of the next operation on st (under g_mu)
clk::time_point next_start(Stream* s) { return std::max(s->done, clk::now()); }

void wait_until(clk::time_point t) {
    while (clk::now() < t) std::this_thread::sleep_for(std::chrono::microseconds(20));
}

void* alloc(size_t n, hipMemoryType type) {
    const size_t bytes = ((std::max<size_t>(n, 1) + 255) / 256) * 256;
    void* p = aligned_alloc(256, bytes);
    if (!p) return nullptr;
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    g_allocs[(uintptr_t)p] = {bytes, type};
    return p;
}

hipError_t release(void* p, hipMemoryType type) {
    if (!p) return hipSuccess;
    {
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        auto it = g_allocs.find((uintptr_t)p);
        if (it == g_allocs.end() || it->second.second != type) return hipErrorInvalidValue;
        check_write(nullptr, clk::now(), it->first, it->first + it->second.first, "free");
        g_allocs.erase(it);
    }
    free(p);
    return hipSuccess;
}

// ---------------------------------------------------------------------------------------------- kernels

// c * b from the kernel's split tables (gf_kernels.hpp CoefTab): T0[b & 7] ^ T1[(b >> 3) & 7] ^ T2[b >> 6]
inline uint8_t tab_mul(const CoefTab& t, uint8_t b) {
    auto byte = [](uint32_t w, int i) { return (uint8_t)(w >> (8 * i)); };
    const int e0 = b & 7, e1 = (b >> 3) & 7, e2 = b >> 6;
    const uint8_t x0 = e0 < 4 ? byte(t.t0lo, e0) : byte(t.t0hi, e0 - 4);
    const uint8_t x1 = e1 < 4 ? byte(t.t1lo, e1) : byte(t.t1hi, e1 - 4);
    return x0 ^ x1 ^ byte(t.t2, e2);
}

inline uint8_t fold(const CoefTab& t, uint8_t x, bool bin) { return bin ? (uint8_t)(x & (uint8_t)t.mask) : tab_mul(t, x); }

// the kernel's workgroup -> (launch stripe, chunk) map (gf_kernels.hip wg_coords)
void wg_coords(const GfLaunch& a, long long b, unsigned grid_x, int& s, int& w) {
    if (a.grid_map == 1) {
        const long long per = (long long)grid_x >> 3;
        b = (b & 7) * per + (b >> 3);
    } else if (a.grid_map == 2) {
        const long long i = b >> 3;
        const long long ls = i / a.wg_per_stripe;
        const long long G = a.map_group;
        s = (int)(((ls / G) * 8 + (b & 7)) * G + ls % G);
        w = (int)(i - ls * a.wg_per_stripe);
        return;
    }
    s = (int)(b / a.wg_per_stripe);
    w = (int)(b - (long long)s * a.wg_per_stripe);
}

int launch_prog(const GfLaunch& a, int mode, int& s) {
    int r = 0;
    if (mode == ecg::GF_MODE_STRIDED && a.row_split) {
        r = s % a.row_split;
        s = s / a.row_split;
    }
    const int p = a.prog_of_stripe ? a.prog_of_stripe[s] : 0;
    return (mode == ecg::GF_MODE_STRIDED && a.row_split) ? p * a.row_split + r : p;
}

const uint8_t* src_ptr(const GfLaunch& a, int mode, int s, int prog, int j) {
    if (mode == ecg::GF_MODE_INLINE || mode == ecg::GF_MODE_INLINE_LAT) return a.isrc[j];
    if (mode == ecg::GF_MODE_PTRS) return a.src_ptrs[(size_t)s * a.k + j];
    const long long sa = a.stripe_of ? a.stripe_of[s] : s;
    return a.in_base + sa * a.in_sstride + (long long)a.src_ids[prog * a.k + j] * a.in_bstride;
}

uint8_t* dst_ptr(const GfLaunch& a, int mode, int s, int prog, int p) {
    if (mode == ecg::GF_MODE_INLINE || mode == ecg::GF_MODE_INLINE_LAT) return a.idst[p];
    if (mode == ecg::GF_MODE_PTRS) return a.dst_ptrs[(size_t)s * a.m + p];
    const long long sa = a.stripe_of ? a.stripe_of[s] : s;
    return a.out_base + sa * a.out_sstride + (long long)a.dst_ids[prog * a.m + p] * a.out_bstride;
}

// one workgroup of gf_vec_kernel (bytes of 16-byte columns [c0, c1)) or gf_byte_kernel (bytes [b0, b1)):
// both computed from whole input bytes first, then stored, like the kernels' register accumulators
struct TabRange {
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    void add(const void* p, size_t n) {
        lo = std::min(lo, (uintptr_t)p);
        hi = std::max(hi, (uintptr_t)p + n);
    }
};

void run_wg(const GfLaunch& a, int mode, int MT, bool bin, bool vec, long long b, unsigned grid_x, int rt,
            TabRange& tr) {
    int s = 0, w = 0;
    wg_coords(a, b, grid_x, s, w);
    const int prog = launch_prog(a, mode, s);
    const int row0 = rt * MT, nrows = std::min(MT, a.m - row0);
    const CoefTab* T = a.tabs + (size_t)(prog * a.rtiles + rt) * (size_t)a.k * MT;
    tr.add(T, (size_t)a.k * MT * sizeof(CoefTab));
    long long lo, hi;
    if (vec) {
        const long long ncols = a.B >> 4, c0 = (long long)w * a.cols_per_wg;
        lo = c0 << 4;
        hi = std::min(c0 + (long long)a.cols_per_wg, ncols) << 4;
    } else {
        lo = a.off0 + (long long)w * a.cols_per_wg;
        hi = std::min(lo + (long long)a.cols_per_wg, a.B);
    }
    if (lo >= hi) return;
    std::vector<uint8_t> acc((size_t)nrows * (hi - lo), 0);
    for (int j = 0; j < a.k; j++) {
        const uint8_t* in = src_ptr(a, mode, s, prog, j);
        for (int p = 0; p < nrows; p++) {
            const CoefTab& t = T[(size_t)j * MT + p];
            uint8_t* o = acc.data() + (size_t)p * (hi - lo);
            for (long long x = lo; x < hi; x++) o[x - lo] ^= fold(t, in[x], bin);
        }
    }
    for (int p = 0; p < nrows; p++) memcpy(dst_ptr(a, mode, s, prog, row0 + p) + lo, acc.data() + (size_t)p * (hi - lo), hi - lo);
}

void post_flag(unsigned* f, unsigned seq) { __atomic_store_n(f, seq, __ATOMIC_RELEASE); }

void emulate_gf(const GfLaunch& a, int mode, int MT, bool bin, bool vec, dim3 g, TabRange& tr) {
    for (unsigned y = 0; y < g.y; y++)
        for (unsigned x = 0; x < g.x; x++) run_wg(a, mode, MT, bin, vec, x, g.x, (int)y, tr);
    if (mode == ecg::GF_MODE_INLINE_LAT && a.done_flags && vec)
        for (unsigned i = 0; i < g.x * g.y; i++) post_flag(a.done_flags + i, a.done_seq);
}

// gf_lat_dword_kernel's argument block (gf_kernels.hip LatArgs<KB, MT>): tabs, done_flags, B, k, m, done_seq,
// src[KB], dst[MT] in declaration order
struct LatHead {
    const CoefTab* tabs;
    unsigned* done_flags;
    long long B;
    int k, m;
    unsigned done_seq;
};

void emulate_lat(const void* argp, int MT, bool bin, int KB, dim3 g, TabRange& tr) {
    LatHead h;
    memcpy(&h, argp, sizeof(h));
    tr.add(h.tabs, (size_t)h.k * MT * sizeof(CoefTab));
    const size_t off = (sizeof(LatHead) + 7) & ~(size_t)7;
    const uint8_t* const* src = reinterpret_cast<const uint8_t* const*>((const char*)argp + off);
    uint8_t* const* dst = reinterpret_cast<uint8_t* const*>((const char*)argp + off + (size_t)KB * sizeof(void*));
    std::vector<uint8_t> acc((size_t)h.m * h.B, 0);
    for (int u = 0; u < h.k; u++)
        for (int p = 0; p < h.m; p++) {
            const CoefTab& t = h.tabs[(size_t)u * MT + p];
            for (long long x = 0; x < h.B; x++) acc[(size_t)p * h.B + x] ^= fold(t, src[u][x], bin);
        }
    for (int p = 0; p < h.m; p++) memcpy(dst[p], acc.data() + (size_t)p * h.B, (size_t)h.B);
    if (h.done_flags)
        for (unsigned i = 0; i < g.x; i++) post_flag(h.done_flags + i, h.done_seq);
}

void emulate_fill(void** args) {
    uint8_t* dst = *(uint8_t**)args[0];
    const long long nbytes = *(long long*)args[1];
    const unsigned long long seed = *(unsigned long long*)args[2], woff = *(unsigned long long*)args[3];
    for (long long w = 0; w < ((nbytes + 7) >> 3); w++) {
        unsigned long long z = seed + (woff + (unsigned long long)w) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (long long b = w * 8; b < std::min(nbytes, w * 8 + 8); ++b) dst[b] = (uint8_t)(z >> (8 * (b - w * 8)));
    }
}

// template arguments of a mangled kernel name after the kernel's own name, in order:
// "..13gf_vec_kernelILi4ELi2ELi3ELb0EEEvNS_8GfLaunchE" -> 4, 2, 3, 0
std::vector<int> template_args(const std::string& mangled, size_t from) {
    std::vector<int> v;
    for (size_t i = from; i < mangled.size(); i++) {
        if (mangled[i] == 'L' && i + 1 < mangled.size() && (mangled[i + 1] == 'i' || mangled[i + 1] == 'b')) {
            size_t j = i + 2;
            const bool neg = j < mangled.size() && mangled[j] == 'n';
            if (neg) j++;
            int x = 0;
            while (j < mangled.size() && mangled[j] >= '0' && mangled[j] <= '9') x = x * 10 + (mangled[j++] - '0');
            v.push_back(neg ? -x : x);
            i = j;
        }
    }
    return v;
}

}  // namespace

// ------------------------------------------------------------------------------------------- runtime API

extern "C" void** __hipRegisterFatBinary(const void*) {
    static void* module = nullptr;
    return &module;
}
extern "C" void __hipUnregisterFatBinary(void**) {}
extern "C" void __hipRegisterFunction(void**, const void* hostFunction, char*, const char* deviceName, unsigned int,
                                      uint3*, uint3*, dim3*, dim3*, int*) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    g_kernels[hostFunction] = deviceName;
}
extern "C" hipError_t __hipPopCallConfiguration(dim3*, dim3*, size_t*, hipStream_t*) { return hipErrorNotSupported; }
// the device code object this stand-in replaces (tools/tsan_host.sh points the kernel file's fat-binary
// symbol here)
extern "C" const char hip_stub_fatbin[16] = {0};

hipError_t hipLaunchKernel(const void* f, dim3 g, dim3 blk, void** args, size_t, hipStream_t st) {
    std::string name;
    {
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        auto it = g_kernels.find(f);
        if (it == g_kernels.end()) return hipErrorInvalidDeviceFunction;
        name = it->second;
        if (as_stream(st)->device != t_device) {  // a launch goes to the current device's streams only
            fprintf(stderr, "hip_stub: launch on a stream of device %d while device %d is current\n",
                    as_stream(st)->device, t_device);
            S().hazards++;
            return hipErrorInvalidHandle;
        }
    }
    auto targs = [&](const char* k) { return template_args(name, name.find(k) + strlen(k)); };
    TabRange tr;
    if (noop_mode()) {
        (void)enqueue(st);
        return hipSuccess;
    }
    if (name.find("gf_vec_kernel") != std::string::npos) {  // <MT, MODE, NT, BIN>
        const std::vector<int> t = targs("gf_vec_kernel");
        emulate_gf(*(const GfLaunch*)args[0], t.at(1), t.at(0), t.at(3) != 0, true, g, tr);
    } else if (name.find("gf_byte_kernel") != std::string::npos) {  // <MT, MODE, BIN>
        const std::vector<int> t = targs("gf_byte_kernel");
        emulate_gf(*(const GfLaunch*)args[0], t.at(1), t.at(0), t.at(2) != 0, false, g, tr);
    } else if (name.find("gf_lat_dword_kernel") != std::string::npos) {  // <MT, BIN, KB, EAGER>
        const std::vector<int> t = targs("gf_lat_dword_kernel");
        emulate_lat(args[0], t.at(0), t.at(1) != 0, t.at(2), g, tr);
    } else if (name.find("fill_splitmix_kernel") != std::string::npos) {
        emulate_fill(args);
    } else {
        fprintf(stderr, "hip_stub: kernel %s is not emulated\n", name.c_str());
        return hipErrorNotSupported;
    }
    (void)blk;
    const clk::time_point done = enqueue(st);
    if (tr.hi > tr.lo) {  // the launch reads these tables until it completes
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        g_readers.push_back({tr.lo, tr.hi, as_stream(st), done});
    }
    return hipSuccess;
}

// test hooks for tests/tsan/engine_race.cpp
extern "C" void hip_stub_stall(hipStream_t st, int ms) {  // work worth `ms` of device time queued on st
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    Stream* s = as_stream(st);
    s->done = next_start(s) + std::chrono::milliseconds(ms);
}
extern "C" long hip_stub_hazards() { return S().hazards.load(); }
extern "C" long hip_stub_not_ready() { return S().not_ready.load(); }

hipError_t hipMalloc(void** p, size_t n) {
    *p = alloc(n, hipMemoryTypeDevice);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) { return release(p, hipMemoryTypeDevice); }
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) {
    *p = alloc(n, hipMemoryTypeHost);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void* p) { return release(p, hipMemoryTypeHost); }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) {
    *d = h;
    return hipSuccess;
}
hipError_t hipPointerGetAttributes(hipPointerAttribute_t* at, const void* p) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    auto it = g_allocs.upper_bound((uintptr_t)p);
    if (it == g_allocs.begin()) return hipErrorInvalidValue;
    --it;
    if ((uintptr_t)p >= it->first + it->second.first) return hipErrorInvalidValue;
    memset(at, 0, sizeof(*at));
    at->type = it->second.second;
    at->devicePointer = at->hostPointer = const_cast<void*>(p);
    return hipSuccess;
}

void check_stream_write(hipStream_t st, const void* d, size_t n, const char* what) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    Stream* s = as_stream(st);
    check_write(s, next_start(s), (uintptr_t)d, (uintptr_t)d + n, what);
}

hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t st) {
    check_stream_write(st, d, n, "copy");
    if (n) memmove(d, s, n);
    enqueue(st);
    return hipSuccess;
}
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind k) {
    hipMemcpyAsync(d, s, n, k, nullptr);
    return hipDeviceSynchronize();
}
hipError_t hipMemcpy2DAsync(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, hipMemcpyKind,
                            hipStream_t st) {
    for (size_t r = 0; r < h; r++) memmove((char*)d + r * dp, (const char*)s + r * sp, w);
    enqueue(st);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t st) {
    check_stream_write(st, d, n, "memset");
    memset(d, v, n);
    enqueue(st);
    return hipSuccess;
}

hipError_t hipStreamCreateWithFlags(hipStream_t* st, unsigned int) {
    Stream* s = new Stream();
    s->device = t_device;
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    g_streams.push_back(s);
    *st = reinterpret_cast<hipStream_t>(s);
    return hipSuccess;
}
hipError_t hipStreamCreate(hipStream_t* st) { return hipStreamCreateWithFlags(st, 0); }
hipError_t hipStreamCreateWithPriority(hipStream_t* st, unsigned int f, int) { return hipStreamCreateWithFlags(st, f); }
hipError_t hipStreamDestroy(hipStream_t st) {
    Stream* s = as_stream(st);
    clk::time_point t;
    {
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        t = s->done;
    }
    wait_until(t);  // like the runtime: queued work finishes first
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    g_streams.erase(std::remove(g_streams.begin(), g_streams.end(), s), g_streams.end());
    delete s;
    return hipSuccess;
}
hipError_t hipStreamQuery(hipStream_t st) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (clk::now() >= as_stream(st)->done) return hipSuccess;
    S().not_ready++;
    return hipErrorNotReady;
}
hipError_t hipStreamSynchronize(hipStream_t st) {
    clk::time_point t;
    {
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        t = as_stream(st)->done;
    }
    wait_until(t);
    return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t st, hipEvent_t ev, unsigned int) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    Stream* s = as_stream(st);
    const Event* e = reinterpret_cast<const Event*>(ev);
    if (e->recorded) s->done = std::max(s->done, e->done);
    return hipSuccess;
}
hipError_t hipDeviceSynchronize() {
    clk::time_point t;
    {
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        t = g_null.done;  // the current device's streams
        for (Stream* s : g_streams)
            if (s->device == t_device) t = std::max(t, s->done);
    }
    wait_until(t);
    return hipSuccess;
}

hipError_t hipEventCreateWithFlags(hipEvent_t* ev, unsigned) {
    Event* e = new Event();
    e->device = t_device;
    *ev = reinterpret_cast<hipEvent_t>(e);
    return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* ev) { return hipEventCreateWithFlags(ev, 0); }
hipError_t hipEventDestroy(hipEvent_t ev) {
    delete reinterpret_cast<Event*>(ev);
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t ev, hipStream_t st) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    Event* e = reinterpret_cast<Event*>(ev);
    if (as_stream(st)->device != e->device) {  // an event records on streams of its own device only
        fprintf(stderr, "hip_stub: event of device %d recorded on a stream of device %d\n", e->device,
                as_stream(st)->device);
        S().hazards++;
        return hipErrorInvalidHandle;
    }
    e->done = as_stream(st)->done;
    e->recorded = true;
    return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t ev) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    const Event* e = reinterpret_cast<const Event*>(ev);
    if (!e->recorded || clk::now() >= e->done) return hipSuccess;
    S().not_ready++;
    return hipErrorNotReady;
}
hipError_t hipEventSynchronize(hipEvent_t ev) {
    clk::time_point t;
    {
        std::lock_guard<std::recursive_mutex> lk(g_mu);
        t = reinterpret_cast<const Event*>(ev)->done;
    }
    wait_until(t);
    return hipSuccess;
}

hipError_t hipGetDevice(int* d) {
    *d = t_device;
    return hipSuccess;
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= kDevices) return hipErrorInvalidDevice;
    t_device = d;
    return hipSuccess;
}
hipError_t hipGetDeviceCount(int* n) {
    *n = kDevices;
    return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) {
    *v = 100000;  // the only attribute the library reads: the wall-clock rate in kHz
    return hipSuccess;
}
hipError_t hipDeviceGetStreamPriorityRange(int* least, int* greatest) {
    *least = 0;
    *greatest = -1;
    return hipSuccess;
}
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "hip_stub error"; }
hipError_t hipGetLastError() { return hipSuccess; }
