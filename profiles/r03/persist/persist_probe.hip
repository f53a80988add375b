// Persistent-worker prototype for single calls: does a resident kernel that polls a
// descriptor ring remove the per-call launch floor the reference's one-call-per-stripe pattern pays
// (proxy.cpp:312-349; handle_repair.cpp:249,371-376)?  Standalone: it does not change libecg; it runs the
// product's own calls beside the worker on the same data and compares bytes and times.
//
// Worker (`worker_kernel`): W workgroups of 256 threads stay resident and poll a ring of 256-byte
// descriptors in pinned host memory.  A descriptor is four 64-byte lines, each starting with the call's
// sequence number, written by the host payload first and sequence numbers last, so a line whose sequence
// number is current carries current fields (the worker takes the descriptor only when all four lines
// agree).  A call is RS-style region product, k <= 16 inputs, m <= 8 outputs, 4 bytes per lane, the
// product's v_perm split-table multiply with tables in device memory.  Every workgroup posts a per-call
// flag with the product's release sequence (gf_done_flag.hpp).  Bounded: a worker exits when told to
// (stop line), after `idle_us` without a descriptor, after `life_ms` in total, or after `max_polls` polls,
// whichever comes first; the host relaunches it from the first unfinished sequence number when a call's
// flags do not arrive and the worker's stream is idle.
//
// Host tier (synchronous, zero-copy; config 1's shape): the call gathers its inputs into the descriptor's
// pinned slot, posts the descriptor, polls the flags, scatters the outputs -- the product's host tier
// minus the launch.  Device tier (asynchronous, HBM blocks): descriptors carry HBM pointers and are posted
// back to back; the host only waits for a ring slot's previous call before reusing it.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Ierasure-codes-prototype_amd/csrc profiles/r03/persist/persist_probe.hip
//        -Lerasure-codes-prototype_amd/lib -lecg -lhsa-runtime64 -Wl,-rpath,'$ORIGIN/../erasure-codes-prototype_amd/lib' -o profiles/r03/persist/persist_probe
// Run:   timeout -k 10 120 profiles/r03/persist/persist_probe [calls]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include "ecg.h"
#include "gf256.hpp"
#include "gf_kernels.hpp"

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

using ecg::CoefTab;

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

constexpr int kT = 256;       // threads per worker workgroup (dword columns per workgroup per pass)
constexpr int kMaxW = 64;     // workgroups of a worker (flags per ring slot)
constexpr int kKB = 16;       // inputs per call (padded, masked)
constexpr int kMB = 8;        // outputs per call
constexpr int kSlotsDev = 256;

// descriptor: 4 lines x 16 dwords; dword 0 of every line = sequence number
struct alignas(256) Desc {
    unsigned w[64];
};
// payload positions (dword index; never 0, 16, 32, 48)
constexpr int P_K = 1, P_M = 2, P_B = 3, P_TABS = 4;  // tabs: dwords 4-5
constexpr int in_pos(int j) { return j < 5 ? 6 + 2 * j : j < 12 ? 17 + 2 * (j - 5) : 33 + 2 * (j - 12); }
constexpr int out_pos(int p) { return p < 2 ? 41 + 2 * p : 49 + 2 * (p - 2); }
static_assert(in_pos(4) == 14 && in_pos(5) == 17 && in_pos(11) == 29 && in_pos(12) == 33 && in_pos(15) == 39, "");
static_assert(out_pos(1) == 43 && out_pos(2) == 49 && out_pos(7) == 59, "");

struct Ctl {  // one line in pinned host memory
    unsigned stop;
    unsigned pad[15];
};

#define CONSTP __attribute__((address_space(4)))

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t gmul(const CONSTP CoefTab& t, uint32_t x) {
    const uint32_t i0 = x & 0x07070707u, i1 = (x >> 3) & 0x07070707u, i2 = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(t.t0hi, t.t0lo, i0), __builtin_amdgcn_perm(t.t1hi, t.t1lo, i1),
                                       __builtin_amdgcn_perm(t.t2, t.t2, i2), 0x96);
}

// release of a workgroup's outputs, then its flag (the product's epilogue, csrc/gf_done_flag.hpp)
__device__ __forceinline__ void post_flag(unsigned* flag, unsigned seq) {
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// this workgroup's share of one call described by d (LDS), specialised like the product's latency kernel:
// KB inputs (padded, masked), MB output rows, so an RS(6,4) call multiplies 24 coefficients per dword and
// loads 24 tables, not 128
template <int KB, int MB>
__device__ __forceinline__ void do_call_t(const unsigned* d) {
    const int tid = threadIdx.x;
    const int k = (int)d[P_K], m = (int)d[P_M];
    const long long ndw = (long long)d[P_B] >> 2;
    const CONSTP CoefTab* T = (const CONSTP CoefTab*)(uintptr_t)(((unsigned long long)d[P_TABS + 1] << 32) | d[P_TABS]);
    const uint8_t* in[KB];
    uint8_t* out[MB];
#pragma unroll
    for (int j = 0; j < KB; j++)
        in[j] = (const uint8_t*)(uintptr_t)(((unsigned long long)d[in_pos(j < k ? j : 0) + 1] << 32) | d[in_pos(j < k ? j : 0)]);
#pragma unroll
    for (int p = 0; p < MB; p++) out[p] = (uint8_t*)(uintptr_t)(((unsigned long long)d[out_pos(p) + 1] << 32) | d[out_pos(p)]);
    for (long long c = (long long)blockIdx.x * kT + tid; c < ndw; c += (long long)gridDim.x * kT) {
        uint32_t x[KB];
#pragma unroll
        for (int j = 0; j < KB; j++) x[j] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(in[j]) + c);
        uint32_t acc[MB];
#pragma unroll
        for (int p = 0; p < MB; p++) acc[p] = 0u;
#pragma unroll
        for (int j = 0; j < KB; j++) {
            const uint32_t keep = j < k ? ~0u : 0u;
#pragma unroll
            for (int p = 0; p < MB; p++) acc[p] = __builtin_amdgcn_bitop3_b32(acc[p], gmul(T[j * kMB + p], x[j]), keep, 0x78);
        }
#pragma unroll
        for (int p = 0; p < MB; p++)
            if (p < m) __builtin_nontemporal_store(acc[p], reinterpret_cast<uint32_t*>(out[p]) + c);
    }
}

__device__ __forceinline__ void do_call(const unsigned* d) {
    const unsigned k = d[P_K], m = d[P_M];
    if (k <= 6 && m <= 4) do_call_t<6, 4>(d);
    else if (k <= 10 && m <= 4) do_call_t<10, 4>(d);
    else do_call_t<kKB, kMB>(d);
}

// Workgroup 0 is the leader: it alone polls the ring in host memory (one PCIe round trip per poll) and
// republishes each descriptor it takes into a device-memory mailbox; the other workgroups poll the mailbox
// (L2), so an idle worker costs the link one 256-byte read per poll, not one per workgroup.
// Exit codes written to exit_info[blockIdx.x] (pinned): 1 stop, 2 idle, 3 life, 4 polls, 5 leader exited.
__global__ void __launch_bounds__(kT, 1) worker_kernel(const Desc* ring, int nslots, unsigned* flags, const Ctl* ctl,
                                                       Desc* mbox, unsigned* mbseq, unsigned* mbexit, unsigned start_seq,
                                                       unsigned long long idle_ticks, unsigned long long life_ticks,
                                                       unsigned max_polls, unsigned* exit_info) {
    __shared__ unsigned d[64];
    __shared__ unsigned go;
    const int tid = threadIdx.x;
    const bool leader = blockIdx.x == 0;
    unsigned next = start_seq;
    const unsigned long long t0 = wall_clock64();
    unsigned long long last = t0;
    // followers wait longer than the leader before giving up on their own: the leader's exit tells them
    const unsigned long long my_idle = leader ? idle_ticks : 2 * idle_ticks;
    unsigned why = 4;
    for (unsigned polls = 0; polls < max_polls; polls++) {
        const unsigned slot = next % (unsigned)nslots;
        if (leader) {
            if (tid < 64) {  // wave 0: the whole descriptor and the stop line in one round trip
                const unsigned v = ld_sys(&ring[slot].w[tid]);
                const unsigned stop = ld_sys(&ctl->stop);
                d[tid] = v;
                if (tid == 0) go = stop ? 2u : 0u;
            }
            __syncthreads();
            if (tid == 0 && go == 0 && d[0] == next && d[16] == next && d[32] == next && d[48] == next) go = 1;
            __syncthreads();
            if (go == 1 && gridDim.x > 1 && tid < 64) {  // republish for the followers: payload, then seq
                __hip_atomic_store(&mbox[slot].w[tid], d[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tid == 0) __hip_atomic_store(&mbseq[slot], next, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            if (tid == 0) {
                const unsigned sq = __hip_atomic_load(&mbseq[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned ex = __hip_atomic_load(mbexit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                go = sq == next ? 1u : ex ? 3u : 0u;
            }
            __syncthreads();
            if (go == 1 && tid < 64) d[tid] = __hip_atomic_load(&mbox[slot].w[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
        }
        const unsigned g = go;
        if (g == 2 || g == 3) {
            why = g == 2 ? 1 : 5;
            break;
        }
        if (g == 0) {
            const unsigned long long t = wall_clock64();
            if (t - last > my_idle) {
                why = 2;
                break;
            }
            if (t - t0 > life_ticks) {
                why = 3;
                break;
            }
            __syncthreads();  // d / go are rewritten by the next poll
            continue;
        }
        do_call(d);  // one call over this workgroup's dword columns
        post_flag(flags + (size_t)(next % (unsigned)nslots) * kMaxW + blockIdx.x, next);
        next++;
        last = wall_clock64();
        __syncthreads();
    }
    if (leader && tid == 0) __hip_atomic_store(mbexit, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) __hip_atomic_store(exit_info + blockIdx.x, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Worker {
    hipStream_t st{};
    Desc* ring = nullptr;  // pinned, mapped
    Desc* ring_dev = nullptr;
    unsigned* flags = nullptr;
    unsigned* flags_dev = nullptr;
    Ctl* ctl = nullptr;
    Ctl* ctl_dev = nullptr;
    unsigned* exit_info = nullptr;
    unsigned* exit_dev = nullptr;
    Desc* mbox = nullptr;      // device memory: the leader's copies of the descriptors
    unsigned* mbseq = nullptr;  // device: [nslots] sequence numbers, then the exit word
    double last_active = 0, idle_s = 0;
    int nslots = 0, W = 0;
    unsigned seq = 0;  // last posted
    long long launches = 0, relaunch_waits = 0;
    unsigned long long idle_ticks = 0, life_ticks = 0;
    bool alive = false;

    void init(int slots, int workgroups, double idle_us, double life_ms) {
        nslots = slots;
        W = workgroups;
        CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        CK(hipHostMalloc((void**)&ring, sizeof(Desc) * slots, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostGetDevicePointer((void**)&ring_dev, ring, 0));
        CK(hipHostMalloc((void**)&flags, sizeof(unsigned) * slots * kMaxW, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostGetDevicePointer((void**)&flags_dev, flags, 0));
        CK(hipHostMalloc((void**)&ctl, sizeof(Ctl), hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostGetDevicePointer((void**)&ctl_dev, ctl, 0));
        CK(hipHostMalloc((void**)&exit_info, sizeof(unsigned) * kMaxW, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostGetDevicePointer((void**)&exit_dev, exit_info, 0));
        memset(ring, 0, sizeof(Desc) * slots);
        memset(flags, 0, sizeof(unsigned) * slots * kMaxW);
        memset(ctl, 0, sizeof(Ctl));
        CK(hipMalloc((void**)&mbox, sizeof(Desc) * slots));
        CK(hipMalloc((void**)&mbseq, sizeof(unsigned) * (slots + 1)));
        CK(hipMemset(mbseq, 0, sizeof(unsigned) * (slots + 1)));
        idle_s = idle_us * 1e-6;
        int rate_khz = 0;
        CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
        idle_ticks = (unsigned long long)(idle_us * rate_khz / 1000.0);
        life_ticks = (unsigned long long)(life_ms * rate_khz);
    }
    void launch(unsigned start) {
        memset(exit_info, 0, sizeof(unsigned) * kMaxW);
        CK(hipMemsetAsync(mbseq + nslots, 0, sizeof(unsigned), st));  // exit word of the new generation
        hipLaunchKernelGGL(worker_kernel, dim3(W), dim3(kT), 0, st, ring_dev, nslots, flags_dev, ctl_dev, mbox, mbseq,
                           mbseq + nslots, start, idle_ticks, life_ticks, 1u << 22, exit_dev);
        CK(hipGetLastError());
        launches++;
        alive = true;
        last_active = now();
    }
    // before posting call s: a worker idle for longer than its limit has exited; start a new one at once
    // rather than after a stalled wait
    void ensure(unsigned s) {
        if (now() - last_active > 0.8 * idle_s && hipStreamQuery(st) == hipSuccess) launch(s);
    }
    // descriptor for call `s`: payload first, the four sequence numbers last (x86 stores stay in order)
    void post(unsigned s, int k, int m, unsigned B, const CoefTab* tabs, const uint8_t* const* in, uint8_t* const* out) {
        Desc& d = ring[s % (unsigned)nslots];
        d.w[P_K] = (unsigned)k;
        d.w[P_M] = (unsigned)m;
        d.w[P_B] = B;
        const unsigned long long t = (unsigned long long)(uintptr_t)tabs;
        d.w[P_TABS] = (unsigned)t;
        d.w[P_TABS + 1] = (unsigned)(t >> 32);
        for (int j = 0; j < kKB; j++) {
            const unsigned long long p = (unsigned long long)(uintptr_t)(j < k ? in[j] : in[0]);
            d.w[in_pos(j)] = (unsigned)p;
            d.w[in_pos(j) + 1] = (unsigned)(p >> 32);
        }
        for (int p = 0; p < kMB; p++) {
            const unsigned long long q = (unsigned long long)(uintptr_t)(p < m ? out[p] : out[0]);
            d.w[out_pos(p)] = (unsigned)q;
            d.w[out_pos(p) + 1] = (unsigned)(q >> 32);
        }
        std::atomic_thread_fence(std::memory_order_release);
        for (int l = 0; l < 4; l++) __atomic_store_n(&d.w[16 * l], s, __ATOMIC_RELEASE);
    }
    bool done(unsigned s) const {
        const unsigned* f = flags + (size_t)(s % (unsigned)nslots) * kMaxW;
        for (int w = 0; w < W; w++)
            if (__atomic_load_n(&f[w], __ATOMIC_ACQUIRE) != s) return false;
        return true;
    }
    // wait for call s; if its flags stall and the worker has exited, relaunch it from s
    void wait(unsigned s) {
        const double t0 = now();
        double next_check = t0 + 20e-6;
        while (!done(s)) {
            const double t = now();
            if (t > next_check) {
                next_check = t + 20e-6;
                const hipError_t q = hipStreamQuery(st);
                if (q == hipSuccess) {  // every workgroup of the worker has exited: none can still write
                    if (done(s)) break;
                    relaunch_waits++;
                    launch(s);
                } else if (q != hipErrorNotReady) {
                    fprintf(stderr, "worker stream: %s\n", hipGetErrorString(q));
                    exit(4);
                }
            }
            if (t - t0 > 2.0) {
                fprintf(stderr, "call %u never completed\n", s);
                exit(5);
            }
        }
        last_active = now();
    }
    void stop() {
        __atomic_store_n(&ctl->stop, 1u, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(st));
        ctl->stop = 0;
        alive = false;
        CK(hipFree(mbox));
        CK(hipFree(mbseq));
        CK(hipHostFree(ring));
        CK(hipHostFree(flags));
        CK(hipHostFree(ctl));
        CK(hipHostFree(exit_info));
        CK(hipStreamDestroy(st));
    }
};

static void make_tabs(const std::vector<int>& M, int k, int m, CoefTab* h) {  // [kKB][kMB], c = M[p][j]
    memset(h, 0, sizeof(CoefTab) * kKB * kMB);
    for (int j = 0; j < k; j++)
        for (int p = 0; p < m; p++) {
            const int c = M[(size_t)p * k + j] & 0xff;
            uint8_t e0[8], e1[8], e2[4];
            for (int e = 0; e < 8; e++) {
                e0[e] = (uint8_t)ecg::gf::mul(c, e);
                e1[e] = (uint8_t)ecg::gf::mul(c, e << 3);
            }
            for (int e = 0; e < 4; e++) e2[e] = (uint8_t)ecg::gf::mul(c, e << 6);
            auto pack = [](const uint8_t* b) {
                return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
            };
            CoefTab& t = h[j * kMB + p];
            t.t0lo = pack(e0);
            t.t0hi = pack(e0 + 4);
            t.t1lo = pack(e1);
            t.t1hi = pack(e1 + 4);
            t.t2 = pack(e2);
        }
}

struct Stat {
    double best = 1e9, sum = 0;
    int n = 0;
};

template <class F>
static Stat bench(const char* name, int calls, F fn) {
    for (int i = 0; i < 100; i++) fn();
    Stat s;
    for (int r = 0; r < 5; r++) {
        const double t0 = now();
        for (int i = 0; i < calls / 5; i++) fn();
        const double us = (now() - t0) / (calls / 5) * 1e6;
        s.best = std::min(s.best, us);
        s.sum += us;
        s.n++;
    }
    printf("  %-34s %8.2f us/call best of 5, %8.2f avg\n", name, s.best, s.sum / s.n);
    fflush(stdout);
    return s;
}

// ---------------------------------------------------------------------------------------- host tier
static void host_tier(int k, int m, int B, int calls) {
    printf("host tier RS(%d,%d), %d B blocks (synchronous calls on pageable host buffers)\n", k, m, B);
    int* Mp = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
    std::vector<int> M(Mp, Mp + k * m);
    std::vector<std::vector<uint8_t>> data(k, std::vector<uint8_t>(B)), par(m, std::vector<uint8_t>(B)),
        mine(m, std::vector<uint8_t>(B));
    unsigned x = 12345;
    for (auto& v : data)
        for (auto& b : v) b = (uint8_t)((x = x * 1103515245u + 12345u) >> 16);
    std::vector<char*> p(k + m);
    for (int i = 0; i < k; i++) p[i] = (char*)data[i].data();
    for (int i = 0; i < m; i++) p[k + i] = (char*)par[i].data();
    const Stat prod = bench("product (launch + flags)", calls, [&] {
        if (ecg_jerasure_matrix_encode(k, m, 8, Mp, p.data(), p.data() + k, B) != 0) exit(2);
    });
    // worker: one slot (one call in flight), blocks in the slot's pinned area
    const int W = std::max(1, std::min(kMaxW, (B / 4 + kT - 1) / kT));
    Worker wk;
    wk.init(4, W, 200.0, 100.0);
    uint8_t *stage = nullptr, *stage_dev = nullptr;
    const size_t pitch = ((size_t)B + 255) & ~(size_t)255;
    CK(hipHostMalloc((void**)&stage, pitch * (k + m), hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&stage_dev, stage, 0));
    CoefTab* tabs_d = nullptr;
    std::vector<CoefTab> tabs_h(kKB * kMB);
    make_tabs(M, k, m, tabs_h.data());
    CK(hipMalloc((void**)&tabs_d, sizeof(CoefTab) * kKB * kMB));
    CK(hipMemcpy(tabs_d, tabs_h.data(), sizeof(CoefTab) * kKB * kMB, hipMemcpyHostToDevice));
    std::vector<const uint8_t*> in(k);
    std::vector<uint8_t*> out(m);
    for (int j = 0; j < k; j++) in[j] = stage_dev + pitch * j;
    for (int q = 0; q < m; q++) out[q] = stage_dev + pitch * (k + q);
    auto call = [&](bool copy) {
        const unsigned s = ++wk.seq;
        if (copy)
            for (int j = 0; j < k; j++) memcpy(stage + pitch * j, data[j].data(), B);
        wk.ensure(s);
        wk.post(s, k, m, (unsigned)B, tabs_d, in.data(), out.data());
        wk.wait(s);
        if (copy)
            for (int q = 0; q < m; q++) memcpy(mine[q].data(), stage + pitch * (k + q), B);
    };
    wk.launch(1);
    call(true);
    for (int q = 0; q < m; q++)
        if (memcmp(mine[q].data(), par[q].data(), B)) {
            fprintf(stderr, "worker parity %d differs from the product's\n", q);
            exit(6);
        }
    const Stat w = bench("persistent worker (gather+post+flags+scatter)", calls, [&] { call(true); });
    bench("persistent worker, no gather/scatter", calls, [&] { call(false); });
    // after an idle gap longer than the worker's idle limit: it has exited, the call relaunches it
    const long long l0 = wk.launches;
    double gap_sum = 0;
    for (int i = 0; i < 50; i++) {
        std::this_thread::sleep_for(std::chrono::microseconds(400));
        const double t0 = now();
        call(true);
        gap_sum += now() - t0;
    }
    printf("  %-34s %8.2f us/call avg (%lld relaunches for 50 calls)\n", "worker after a 400 us idle gap", gap_sum / 50 * 1e6,
           wk.launches - l0);
    fflush(stdout);
    for (int q = 0; q < m; q++)
        if (memcmp(mine[q].data(), par[q].data(), B)) {
            fprintf(stderr, "worker parity %d differs from the product's\n", q);
            exit(6);
        }
    const unsigned why = wk.exit_info[0];
    wk.stop();
    printf("  -> worker %.2f us vs product %.2f us (best): %.2fx; worker launches %lld, relaunch waits %lld, last exit %u\n",
           w.best, prod.best, prod.best / w.best, wk.launches, wk.relaunch_waits, why);
    fflush(stdout);
    CK(hipFree(tabs_d));
    CK(hipHostFree(stage));
    ecg_free(Mp);
}

// ---------------------------------------------------------------------------------------- device tier
// Does a resident worker block other streams?  HIP maps streams onto a few hardware queues
// (GPU_MAX_HW_QUEUES, 4 by default); a kernel that stays resident on a queue shared with another stream
// would hold that stream's work behind it until the worker exits.  With a worker alive (idle limit 30 ms),
// an empty kernel is launched on each of 8 fresh streams and timed to completion; a blocked stream shows
// up as ~30 ms.  Once with the worker on a normal stream, once on a high-priority stream.
__global__ void nop_kernel() {}

static void queue_interference(int priority) {
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    Worker wk;
    wk.init(4, 1, 30000.0, 200.0);
    if (priority) {
        CK(hipStreamDestroy(wk.st));
        CK(hipStreamCreateWithPriority(&wk.st, hipStreamNonBlocking, hi));
    }
    std::vector<hipStream_t> ss(8);
    for (auto& x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    for (auto& x : ss) {  // warm the streams before the worker exists
        hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, x);
        CK(hipStreamSynchronize(x));
    }
    wk.launch(1);
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    printf("worker on a %s stream (priority range %d..%d): empty kernel on 8 other streams, us to completion:",
           priority ? "high-priority" : "normal", lo, hi);
    for (auto& x : ss) {
        const double t0 = now();
        hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, x);
        CK(hipStreamSynchronize(x));
        printf(" %.0f", (now() - t0) * 1e6);
    }
    const hipError_t alive = hipStreamQuery(wk.st);
    printf("; worker still resident: %s\n", alive == hipErrorNotReady ? "yes" : "no");
    fflush(stdout);
    wk.stop();
    for (auto& x : ss) CK(hipStreamDestroy(x));
}

static void device_tier(int k, int m, int B, int S) {
    printf("device tier RS(%d,%d), %d B blocks, %d per-stripe calls on HBM (asynchronous)\n", k, m, B, S);
    int* Mp = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
    std::vector<int> M(Mp, Mp + k * m);
    const int n = k + m;
    uint8_t *st = nullptr, *ref = nullptr;
    CK(hipMalloc((void**)&st, (size_t)S * n * B));
    CK(hipMalloc((void**)&ref, (size_t)S * m * B));
    if (ecg_fill_random(st, (long long)S * n * B, 0x9E5, 0, nullptr) != 0) exit(2);
    hipStream_t s0;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    std::vector<char*> blk(n);
    auto product_pass = [&](uint8_t* outbase) {
        for (int s = 0; s < S; s++) {
            for (int j = 0; j < k; j++) blk[j] = (char*)st + ((size_t)s * n + j) * B;
            for (int q = 0; q < m; q++) blk[k + q] = (char*)outbase + ((size_t)s * m + q) * B;
            if (ecg_dev_matrix_encode(k, m, Mp, blk.data(), blk.data() + k, B, s0) != 0) exit(2);
        }
    };
    product_pass(ref);
    CK(hipStreamSynchronize(s0));
    double best_prod = 1e9;
    for (int r = 0; r < 3; r++) {
        const double t0 = now();
        product_pass(ref);
        CK(hipStreamSynchronize(s0));
        best_prod = std::min(best_prod, now() - t0);
    }
    const double gib = (double)S * k * B / (1 << 30);
    printf("  %-34s %8.1f GiB/s (%.2f us per call)\n", "product (one launch per call)", gib / best_prod, best_prod / S * 1e6);
    const int W = std::max(1, std::min(kMaxW, (B / 4 + kT - 1) / kT));
    Worker wk;
    wk.init(kSlotsDev, W, 200.0, 100.0);
    CoefTab* tabs_d = nullptr;
    std::vector<CoefTab> tabs_h(kKB * kMB);
    make_tabs(M, k, m, tabs_h.data());
    CK(hipMalloc((void**)&tabs_d, sizeof(CoefTab) * kKB * kMB));
    CK(hipMemcpy(tabs_d, tabs_h.data(), sizeof(CoefTab) * kKB * kMB, hipMemcpyHostToDevice));
    uint8_t* mine = nullptr;
    CK(hipMalloc((void**)&mine, (size_t)S * m * B));
    CK(hipMemset(mine, 0, (size_t)S * m * B));
    CK(hipDeviceSynchronize());
    std::vector<const uint8_t*> in(k);
    std::vector<uint8_t*> out(m);
    auto worker_pass = [&]() {
        unsigned first = wk.seq + 1;
        for (int s = 0; s < S; s++) {
            const unsigned q = ++wk.seq;
            if (q >= first + (unsigned)kSlotsDev) wk.wait(q - kSlotsDev);  // the slot's previous call
            for (int j = 0; j < k; j++) in[j] = st + ((size_t)s * n + j) * B;
            for (int p = 0; p < m; p++) out[p] = mine + ((size_t)s * m + p) * B;
            wk.post(q, k, m, (unsigned)B, tabs_d, in.data(), out.data());
        }
        for (unsigned q = (wk.seq >= (unsigned)kSlotsDev ? wk.seq - kSlotsDev + 1 : 1); q <= wk.seq; q++)
            if (q >= first) wk.wait(q);
    };
    wk.launch(1);
    worker_pass();
    double best_w = 1e9;
    for (int r = 0; r < 3; r++) {
        const double t0 = now();
        worker_pass();
        best_w = std::min(best_w, now() - t0);
    }
    std::vector<uint8_t> a((size_t)S * m * B), b((size_t)S * m * B);
    CK(hipMemcpy(a.data(), ref, a.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), mine, b.size(), hipMemcpyDeviceToHost));
    const bool same = a == b;
    wk.stop();
    printf("  %-34s %8.1f GiB/s (%.2f us per call), bytes %s; worker launches %lld, relaunch waits %lld\n",
           "persistent worker (posted back to back)", gib / best_w, best_w / S * 1e6, same ? "identical" : "DIFFER",
           wk.launches, wk.relaunch_waits);
    if (!same) exit(7);
    CK(hipFree(mine));
    CK(hipFree(tabs_d));
    CK(hipFree(st));
    CK(hipFree(ref));
    ecg_free(Mp);
}

// ---------------------------------------------------------------------------------------- BAR variants
// The host writes a small call's inputs (and the worker's descriptors) straight into HBM through the
// large-BAR mapping of a CPU-accessible fine-grained device pool (tools/bar_probe: 6 KiB + sfence in
// ~0.5 us), so the GPU reads them from HBM instead of over PCIe; outputs and flags still go to pinned host
// memory.  Two forms: a launch per call (the product's latency kernel shape) and a resident worker that
// polls the descriptor ring in HBM (each workgroup on its own: an HBM poll costs the link nothing).

__global__ void __launch_bounds__(kT, 1) bar_launch_kernel(const Desc desc, unsigned* flags, unsigned seq) {
    __shared__ unsigned d[64];
    if (threadIdx.x < 64) d[threadIdx.x] = desc.w[threadIdx.x];
    __syncthreads();
    do_call(d);
    post_flag(flags + blockIdx.x, seq);
}

// ring and stop word in BAR-mapped HBM (fine-grained: CPU writes are visible to system-scope loads)
__global__ void __launch_bounds__(kT, 1) bar_worker_kernel(const Desc* ring, int nslots, const unsigned* stopw, unsigned* flags,
                                                           unsigned start_seq, unsigned long long idle_ticks,
                                                           unsigned long long life_ticks, unsigned max_polls,
                                                           unsigned* exit_info) {
    __shared__ unsigned d[64];
    __shared__ unsigned go;
    const int tid = threadIdx.x;
    unsigned next = start_seq;
    const unsigned long long t0 = wall_clock64();
    unsigned long long last = t0;
    unsigned why = 4;
    for (unsigned polls = 0; polls < max_polls; polls++) {
        const unsigned slot = next % (unsigned)nslots;
        if (tid < 64) {
            d[tid] = ld_sys(&ring[slot].w[tid]);
            if (tid == 0) go = ld_sys(stopw) ? 2u : 0u;
        }
        __syncthreads();
        if (tid == 0 && go == 0 && d[0] == next && d[16] == next && d[32] == next && d[48] == next) go = 1;
        __syncthreads();
        const unsigned g = go;
        if (g == 2) {
            why = 1;
            break;
        }
        if (g == 0) {
            const unsigned long long t = wall_clock64();
            if (t - last > idle_ticks) {
                why = 2;
                break;
            }
            if (t - t0 > life_ticks) {
                why = 3;
                break;
            }
            __syncthreads();
            continue;
        }
        do_call(d);
        post_flag(flags + (size_t)slot * kMaxW + blockIdx.x, next);
        next++;
        last = wall_clock64();
        __syncthreads();
    }
    if (tid == 0) __hip_atomic_store(exit_info + blockIdx.x, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct BarMem {  // a CPU-accessible fine-grained HBM pool (HSA), or nothing
    hsa_agent_t cpu{}, gpu{};
    hsa_amd_memory_pool_t pool{};
    bool ok = false;
    void init() {
        if (hsa_init() != HSA_STATUS_SUCCESS) return;
        struct A {
            hsa_agent_t cpu{}, gpu{};
            bool c = false, g = false;
        } a;
        hsa_iterate_agents([](hsa_agent_t x, void* d) {
            A& a = *(A*)d;
            hsa_device_type_t t;
            hsa_agent_get_info(x, HSA_AGENT_INFO_DEVICE, &t);
            if (t == HSA_DEVICE_TYPE_CPU && !a.c) a.cpu = x, a.c = true;
            if (t == HSA_DEVICE_TYPE_GPU && !a.g) a.gpu = x, a.g = true;
            return HSA_STATUS_SUCCESS;
        }, &a);
        if (!a.c || !a.g) return;
        cpu = a.cpu;
        gpu = a.gpu;
        struct P {
            hsa_agent_t cpu;
            hsa_amd_memory_pool_t pool{};
            bool found = false;
        } pp{cpu};
        hsa_amd_agent_iterate_memory_pools(gpu, [](hsa_amd_memory_pool_t q, void* d) {
            P& pp = *(P*)d;
            hsa_amd_segment_t seg;
            uint32_t fl = 0;
            bool alloc = false;
            hsa_amd_memory_pool_access_t acc;
            hsa_amd_memory_pool_get_info(q, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
            hsa_amd_memory_pool_get_info(q, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
            hsa_amd_memory_pool_get_info(q, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
            hsa_amd_agent_memory_pool_get_info(pp.cpu, q, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc);
            if (!pp.found && seg == HSA_AMD_SEGMENT_GLOBAL && alloc && acc != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED &&
                (fl & (HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED | HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_EXTENDED_SCOPE_FINE_GRAINED))) {
                pp.pool = q;
                pp.found = true;
            }
            return HSA_STATUS_SUCCESS;
        }, &pp);
        pool = pp.pool;
        ok = pp.found;
    }
    void* alloc(size_t n) {
        void* p = nullptr;
        if (hsa_amd_memory_pool_allocate(pool, n, 0, &p) != HSA_STATUS_SUCCESS) return nullptr;
        hsa_agent_t both[2] = {gpu, cpu};
        if (hsa_amd_agents_allow_access(2, both, nullptr, p) != HSA_STATUS_SUCCESS) return nullptr;
        return p;
    }
};

static void bar_tier(BarMem& bar, int k, int m, int B, int calls) {
    printf("BAR staging RS(%d,%d), %d B blocks (host writes the inputs into HBM; outputs + flags in pinned host)\n", k, m, B);
    int* Mp = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
    std::vector<int> M(Mp, Mp + k * m);
    std::vector<std::vector<uint8_t>> data(k, std::vector<uint8_t>(B)), par(m, std::vector<uint8_t>(B)),
        mine(m, std::vector<uint8_t>(B));
    unsigned x = 777;
    for (auto& v : data)
        for (auto& b : v) b = (uint8_t)((x = x * 1103515245u + 12345u) >> 16);
    std::vector<char*> p(k + m);
    for (int i = 0; i < k; i++) p[i] = (char*)data[i].data();
    for (int i = 0; i < m; i++) p[k + i] = (char*)par[i].data();
    const Stat prod = bench("product (zero-copy over PCIe)", calls, [&] {
        if (ecg_jerasure_matrix_encode(k, m, 8, Mp, p.data(), p.data() + k, B) != 0) exit(2);
    });
    const int W = std::max(1, std::min(kMaxW, (B / 4 + kT - 1) / kT));
    const size_t pitch = ((size_t)B + 255) & ~(size_t)255;
    constexpr int kBarSlots = 4;
    // HBM (BAR): [kBarSlots] descriptors, a stop line, [kBarSlots][k][pitch] inputs
    uint8_t* hbm = (uint8_t*)bar.alloc(sizeof(Desc) * (kBarSlots + 1) + (size_t)kBarSlots * k * pitch);
    if (!hbm) {
        printf("  BAR allocation failed\n");
        return;
    }
    Desc* ring = (Desc*)hbm;
    unsigned* stopw = (unsigned*)(hbm + sizeof(Desc) * kBarSlots);
    uint8_t* inb = hbm + sizeof(Desc) * (kBarSlots + 1);
    memset(hbm, 0, sizeof(Desc) * (kBarSlots + 1));
    _mm_sfence();
    uint8_t *outh = nullptr, *outd = nullptr;
    CK(hipHostMalloc((void**)&outh, (size_t)kBarSlots * m * pitch, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&outd, outh, 0));
    unsigned *flags = nullptr, *flags_d = nullptr, *exit_info = nullptr, *exit_d = nullptr;
    CK(hipHostMalloc((void**)&flags, sizeof(unsigned) * kBarSlots * kMaxW, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&flags_d, flags, 0));
    CK(hipHostMalloc((void**)&exit_info, sizeof(unsigned) * kMaxW, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&exit_d, exit_info, 0));
    memset(flags, 0, sizeof(unsigned) * kBarSlots * kMaxW);
    CoefTab* tabs_d = nullptr;
    std::vector<CoefTab> tabs_h(kKB * kMB);
    make_tabs(M, k, m, tabs_h.data());
    CK(hipMalloc((void**)&tabs_d, sizeof(CoefTab) * kKB * kMB));
    CK(hipMemcpy(tabs_d, tabs_h.data(), sizeof(CoefTab) * kKB * kMB, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    unsigned seq = 0;
    auto fill = [&](Desc& d, unsigned slot) {
        d.w[P_K] = (unsigned)k;
        d.w[P_M] = (unsigned)m;
        d.w[P_B] = (unsigned)B;
        const unsigned long long t = (unsigned long long)(uintptr_t)tabs_d;
        d.w[P_TABS] = (unsigned)t;
        d.w[P_TABS + 1] = (unsigned)(t >> 32);
        for (int j = 0; j < kKB; j++) {
            const unsigned long long q = (unsigned long long)(uintptr_t)(inb + ((size_t)slot * k + (j < k ? j : 0)) * pitch);
            d.w[in_pos(j)] = (unsigned)q;
            d.w[in_pos(j) + 1] = (unsigned)(q >> 32);
        }
        for (int q = 0; q < kMB; q++) {
            const unsigned long long r = (unsigned long long)(uintptr_t)(outd + ((size_t)slot * m + (q < m ? q : 0)) * pitch);
            d.w[out_pos(q)] = (unsigned)r;
            d.w[out_pos(q) + 1] = (unsigned)(r >> 32);
        }
    };
    auto wait_flags = [&](unsigned slot, unsigned s) {
        const double t0 = now();
        for (int w = 0; w < W; w++)
            while (__atomic_load_n(&flags[slot * kMaxW + w], __ATOMIC_ACQUIRE) != s)
                if (now() - t0 > 2.0) {
                    fprintf(stderr, "BAR call %u: flag never arrived\n", s);
                    exit(8);
                }
    };
    auto gather = [&](unsigned slot) {
        for (int j = 0; j < k; j++) memcpy(inb + ((size_t)slot * k + j) * pitch, data[j].data(), B);
        _mm_sfence();
    };
    auto scatter = [&](unsigned slot) {
        for (int q = 0; q < m; q++) memcpy(mine[q].data(), outh + ((size_t)slot * m + q) * pitch, B);
    };
    auto check = [&](const char* what) {
        for (int q = 0; q < m; q++)
            if (memcmp(mine[q].data(), par[q].data(), B)) {
                fprintf(stderr, "%s: parity %d differs from the product's\n", what, q);
                exit(9);
            }
    };
    // (1) a launch per call, inputs from HBM
    Desc ld{};
    auto launch_call = [&] {
        const unsigned s = ++seq, slot = s % kBarSlots;
        gather(slot);
        fill(ld, slot);
        hipLaunchKernelGGL(bar_launch_kernel, dim3(W), dim3(kT), 0, st, ld, flags_d + slot * kMaxW, s);
        wait_flags(slot, s);
        scatter(slot);
    };
    // inputs change between calls: a stale line of an earlier call's inputs would show here
    auto varying = [&](const char* what, auto&& fn) {
        for (int i = 0; i < 300; i++) {
            for (int j = 0; j < k; j++)
                for (int b = (i * 7) % 64; b < B; b += 61) data[j][b] = (uint8_t)((x = x * 1103515245u + 12345u) >> 16);
            if (ecg_jerasure_matrix_encode(k, m, 8, Mp, p.data(), p.data() + k, B) != 0) exit(2);
            fn();
            check(what);
        }
    };
    launch_call();
    check("BAR launch");
    varying("BAR launch, varying inputs", launch_call);
    const Stat la = bench("launch per call, inputs via BAR", calls, launch_call);
    CK(hipStreamSynchronize(st));
    // (2) a resident worker polling the ring in HBM
    long long launches = 0;
    double last_active = 0;
    const double idle_s = 200e-6;
    auto wlaunch = [&](unsigned start) {
        memset(exit_info, 0, sizeof(unsigned) * kMaxW);
        hipLaunchKernelGGL(bar_worker_kernel, dim3(W), dim3(kT), 0, st, ring, kBarSlots, stopw, flags_d, start,
                           (unsigned long long)(idle_s * 1e6 * rate_khz / 1000.0), (unsigned long long)(100.0 * rate_khz),
                           1u << 24, exit_d);
        CK(hipGetLastError());
        launches++;
        last_active = now();
    };
    int mode = 0;  // 0 full call; 1 empty call (descriptor + flag only); 2 outputs to HBM instead of host memory
    uint8_t* out_hbm = nullptr;
    CK(hipMalloc((void**)&out_hbm, (size_t)kBarSlots * m * pitch));
    auto worker_call = [&] {
        const unsigned s = ++seq, slot = s % kBarSlots;
        if (now() - last_active > 0.8 * idle_s && hipStreamQuery(st) == hipSuccess) wlaunch(s);
        if (mode != 1) gather(slot);
        Desc& d = ring[slot];
        Desc tmp{};
        fill(tmp, slot);
        if (mode == 1) tmp.w[P_B] = 0;
        if (mode == 2)
            for (int q = 0; q < kMB; q++) {
                const unsigned long long r = (unsigned long long)(uintptr_t)(out_hbm + ((size_t)slot * m + (q < m ? q : 0)) * pitch);
                tmp.w[out_pos(q)] = (unsigned)r;
                tmp.w[out_pos(q) + 1] = (unsigned)(r >> 32);
            }
        for (int i = 0; i < 64; i++)
            if (i % 16) d.w[i] = tmp.w[i];
        _mm_sfence();  // payload before the sequence numbers (write-combining stores are not ordered)
        for (int l = 0; l < 4; l++) d.w[16 * l] = s;
        _mm_sfence();
        const double t0 = now();
        double next_check = t0 + 20e-6;
        for (int w = 0; w < W; w++)
            while (__atomic_load_n(&flags[slot * kMaxW + w], __ATOMIC_ACQUIRE) != s) {
                const double t = now();
                if (t > next_check) {
                    next_check = t + 20e-6;
                    if (hipStreamQuery(st) == hipSuccess) {
                        bool all = true;
                        for (int v = 0; v < W; v++) all &= __atomic_load_n(&flags[slot * kMaxW + v], __ATOMIC_ACQUIRE) == s;
                        if (!all) wlaunch(s);
                    }
                }
                if (t - t0 > 2.0) {
                    fprintf(stderr, "BAR worker call %u never completed\n", s);
                    exit(10);
                }
            }
        last_active = now();
        if (mode == 0) scatter(slot);
    };
    wlaunch(seq + 1);
    worker_call();
    check("BAR worker");
    varying("BAR worker, varying inputs", worker_call);
    const Stat wk = bench("resident worker, inputs + ring via BAR", calls, worker_call);
    check("BAR worker");
    mode = 1;
    bench("  same worker, empty call (ring + flag)", calls, worker_call);
    mode = 2;
    bench("  same worker, outputs to HBM", calls, worker_call);
    mode = 0;
    // launch floor for comparison: an empty launch of the same kernel completing by flag
    Desc e0{};
    fill(e0, 0);
    e0.w[P_B] = 0;
    bench("  launch, empty call (flag only)", calls, [&] {
        const unsigned s = ++seq, slot = s % kBarSlots;
        hipLaunchKernelGGL(bar_launch_kernel, dim3(W), dim3(kT), 0, st, e0, flags_d + slot * kMaxW, s);
        wait_flags(slot, s);
    });
    CK(hipFree(out_hbm));
    *stopw = 1;
    _mm_sfence();
    CK(hipStreamSynchronize(st));
    printf("  -> BAR launch %.2f us, BAR worker %.2f us, product %.2f us (best); worker launches %lld, last exit %u\n", la.best,
           wk.best, prod.best, launches, exit_info[0]);
    fflush(stdout);
    CK(hipStreamDestroy(st));
    CK(hipFree(tabs_d));
    CK(hipHostFree(outh));
    CK(hipHostFree(flags));
    CK(hipHostFree(exit_info));
    hsa_amd_memory_pool_free(hbm);
    ecg_free(Mp);
}

int main(int argc, char** argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 4000;
    const bool only_bar = argc > 2 && !strcmp(argv[2], "bar");
    CK(hipSetDevice(0));
    BarMem bar;
    bar.init();
    printf("CPU-accessible fine-grained HBM pool: %s\n", bar.ok ? "yes" : "no");
    if (bar.ok && !(argc > 2 && !strcmp(argv[2], "queues"))) {
        bar_tier(bar, 6, 4, 1024, calls);
        bar_tier(bar, 10, 4, 4096, calls);
        bar_tier(bar, 10, 4, 16 * 1024, calls / 2);
    }
    if (only_bar) return 0;
    if (argc > 2 && !strcmp(argv[2], "queues")) {
        queue_interference(0);
        queue_interference(1);
        return 0;
    }
    host_tier(6, 4, 1024, calls);
    host_tier(10, 4, 16 * 1024, calls / 2);
    host_tier(10, 4, 64 * 1024, calls / 4);
    device_tier(10, 4, 64 * 1024, 4096);
    device_tier(10, 4, 256 * 1024, 1024);
    return 0;
}
