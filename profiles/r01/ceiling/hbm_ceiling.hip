// HBM streaming ceilings on MI355X for the access patterns of the erasure-coding path (tuning tool,
// not shipped).  Pure data movement, no GF arithmetic: what the engine's kernels would reach if the
// multiply were free.  Every pattern reads/writes 16 B per lane per instruction (global_load_dwordx4
// nt / global_store_dwordx4 nt), working sets >> the 256 MiB Infinity Cache.
//
//   read1        one stream, XOR-reduced per lane, one 16 B store per lane at the end (reads only)
//   write1       one stream of stores (writes only)
//   copy         1 -> 1
//   xor_k_m      the engine's stripe layout [S][k+m][B]: k read streams B apart, m written streams
//                (out_p = XOR of the k inputs): the encode access pattern without the multiply
//
// Each lane owns one 16-byte column of a 2 KiB chunk (128-thread workgroups, the engine's shape) or,
// with IN_FLIGHT > 1, IN_FLIGHT consecutive 2 KiB chunks whose loads are all issued before any use.
// Build: hipcc -O3 --offload-arch=gfx950 -o hbm_ceiling profiles/r01/ceiling/hbm_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int TPB = 128;

__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, p); }

// XCD-contiguous workgroup map (the engine's grid_map 1): b % 8 names the XCD.
__device__ __forceinline__ long long xcd_map(long long b) {
    const long long per = (long long)gridDim.x >> 3;
    return (b & 7) * per + (b >> 3);
}

template <int U>
__global__ void __launch_bounds__(TPB) read1(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
    const long long w = xcd_map(blockIdx.x);
    const long long base = w * U * TPB + threadIdx.x;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(in + base + (long long)u * TPB);
    u32x4 a = x[0];
#pragma unroll
    for (int u = 1; u < U; ++u) a ^= x[u];
    if ((a.x & a.y & a.z & a.w) == 0x12345678u) out[threadIdx.x] = a;  // keeps the loads live
}

template <int U>
__global__ void __launch_bounds__(TPB) write1(u32x4* __restrict__ out) {
    const long long w = xcd_map(blockIdx.x);
    const long long base = w * U * TPB + threadIdx.x;
    u32x4 v = {(uint32_t)base, 1u, 2u, 3u};
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + base + (long long)u * TPB, v);
}

template <int U>
__global__ void __launch_bounds__(TPB) copy1(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
    const long long w = xcd_map(blockIdx.x);
    const long long base = w * U * TPB + threadIdx.x;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(in + base + (long long)u * TPB);
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + base + (long long)u * TPB, x[u]);
}

// stripes [S][K+M][B]; workgroup = (stripe, 2 KiB chunk); all K loads issued before the first use.
// Address of 16-byte column c of block j of stripe s (units of 16 B):
//   s * sp16 + j * bp16 + (c / TPB) * cp16 + c % TPB
// block-contiguous layout: bp16 = block pitch, cp16 = TPB; chunk-interleaved: bp16 = TPB, cp16 = (K+M)*TPB.
template <int K, int M>
__global__ void __launch_bounds__(TPB) xor_km(u32x4* __restrict__ st_base, long long sp16, long long bp16,
                                              long long cp16, int wg_per_stripe) {
    const long long w = xcd_map(blockIdx.x);
    const long long s = w / wg_per_stripe;
    const long long ch = w - s * wg_per_stripe;
    u32x4* sp = st_base + s * sp16 + ch * cp16 + threadIdx.x;
    const long long B16 = bp16;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld(sp + j * B16);
    u32x4 a = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= x[j];
#pragma unroll
    for (int p = 0; p < M; ++p) {
        u32x4 o = a;
        o.x ^= p;
        st(sp + (K + p) * B16, o);
    }
}

// k split across the W waves of a workgroup: wave q loads inputs j = q, q+W, ... of one 1 KiB chunk
// (64 lanes x 16 B), partial results are XOR-reduced through LDS, wave q stores outputs p = q, q+W, ...
template <int K, int M, int W>
__global__ void __launch_bounds__(64 * W) xor_split(u32x4* __restrict__ st_base, long long sp16, long long bp16,
                                                    int wg_per_stripe) {
    __shared__ u32x4 red[W][64];
    const long long w = xcd_map(blockIdx.x);
    const long long s = w / wg_per_stripe;
    const long long ch = w - s * wg_per_stripe;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32x4* sp = st_base + s * sp16 + ch * 64 + lane;
    constexpr int PER = (K + W - 1) / W;
    u32x4 x[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i)
        if (wv + i * W < K) x[i] = ld(sp + (wv + i * W) * bp16);
    u32x4 a = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < PER; ++i)
        if (wv + i * W < K) a ^= x[i];
    red[wv][lane] = a;
    __syncthreads();
    for (int p = wv; p < M; p += W) {
        u32x4 o = red[0][lane];
#pragma unroll
        for (int q = 1; q < W; ++q) o ^= red[q][lane];
        o.x ^= p;
        st(sp + (K + p) * bp16, o);
    }
}

// Two sequential streams at a read:write ratio R:W: workgroup u reads R x 2 KiB contiguous from `in`
// at u*R*2K and writes W x 2 KiB contiguous to `out` at u*W*2K (the encode's 10:4 mix, no stripes).
template <int R, int W>
__global__ void __launch_bounds__(TPB) rw_ratio(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
    const long long u = xcd_map(blockIdx.x);
    const u32x4* ip = in + u * R * TPB + threadIdx.x;
    u32x4* op = out + u * W * TPB + threadIdx.x;
    u32x4 x[R];
#pragma unroll
    for (int j = 0; j < R; ++j) x[j] = ld(ip + j * TPB);
    u32x4 a = x[0];
#pragma unroll
    for (int j = 1; j < R; ++j) a ^= x[j];
    if constexpr (W == 0) {
        if ((a.x & a.y & a.z & a.w) == 0x12345678u) out[threadIdx.x] = a;
    } else {
#pragma unroll
        for (int p = 0; p < W; ++p) {
            u32x4 o = a;
            o.x ^= p;
            st(op + p * TPB, o);
        }
    }
}

// Stripe layout [S][K+M][B], K loads per lane, no stores (read side of the encode shape alone).
template <int K, int M>
__global__ void __launch_bounds__(TPB) stripe_read_only(const u32x4* __restrict__ st_base, u32x4* __restrict__ sink,
                                                        long long B16, int wg_per_stripe) {
    const long long w = xcd_map(blockIdx.x);
    const long long s = w / wg_per_stripe;
    const long long ch = w - s * wg_per_stripe;
    const u32x4* sp = st_base + s * (K + M) * B16 + ch * TPB + threadIdx.x;
    u32x4 a = ld(sp);
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= ld(sp + j * B16);
    if ((a.x & a.y & a.z & a.w) == 0x12345678u) sink[threadIdx.x] = a;
}

// Read/write phasing: every workgroup of a resident grid first reads J chunk-jobs (10 inputs each,
// XOR-folded into registers), then writes their 4 outputs; one launch per slice of G*J jobs, so the
// whole chip reads, then writes, then the next launch starts (kernel boundary = global barrier).
template <int J>
__global__ void __launch_bounds__(TPB) phased_10_4(u32x4* __restrict__ st_base, long long B16, int wg_per_stripe,
                                                   long long job0) {
    constexpr int K = 10, M = 4;
    u32x4 acc[J];
    u32x4* sp[J];
#pragma unroll
    for (int i = 0; i < J; ++i) {
        const long long job = job0 + (long long)blockIdx.x * J + i;
        const long long s = job / wg_per_stripe, ch = job - s * wg_per_stripe;
        sp[i] = st_base + s * (K + M) * B16 + ch * TPB + threadIdx.x;
        u32x4 a = ld(sp[i]);
#pragma unroll
        for (int j = 1; j < K; ++j) a ^= ld(sp[i] + j * B16);
        acc[i] = a;
    }
#pragma unroll
    for (int i = 0; i < J; ++i)
#pragma unroll
        for (int p = 0; p < M; ++p) {
            u32x4 o = acc[i];
            o.x ^= p;
            st(sp[i] + (K + p) * B16, o);
        }
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    template <typename F>
    float med_ms(F f, int reps) {
        f();
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a));
            f();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    }
};

static void report(const char* name, double bytes, float ms) {
    const double gbs = bytes / (ms * 1e-3) / 1e9;
    printf("%-34s %8.3f ms  %8.1f GB/s  (%5.1f%% of 8 TB/s)\n", name, ms, gbs, gbs / 80.0);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 7;
    const bool only_new = argc > 2 && atoi(argv[2]) == 1;  // 1: only the phasing experiment
    const long long B = 1ll << 20, S = 4096, K = 10, M = 4;
    const long long total = S * (K + M) * B;  // 56 GiB, the config-2 working set
    u32x4* buf;
    CK(hipMalloc(&buf, total));
    CK(hipMemset(buf, 0x5a, total));
    u32x4* sink;
    CK(hipMalloc(&sink, 4096));
    Timer T;
    const long long half = total / 2;                 // 28 GiB
    const long long n16 = half / 16;
    const u32x4* src = buf;
    u32x4* dst = buf + n16;
    if (!only_new) {
    for (int u : {1, 2, 4, 8}) {
        const long long wgs = n16 / ((long long)u * TPB);
        char nm[64];
        float ms;
        switch (u) {
            case 1: ms = T.med_ms([&] { read1<1><<<wgs, TPB>>>(src, sink); }, reps); break;
            case 2: ms = T.med_ms([&] { read1<2><<<wgs, TPB>>>(src, sink); }, reps); break;
            case 4: ms = T.med_ms([&] { read1<4><<<wgs, TPB>>>(src, sink); }, reps); break;
            default: ms = T.med_ms([&] { read1<8><<<wgs, TPB>>>(src, sink); }, reps); break;
        }
        snprintf(nm, sizeof nm, "read-only  x%d in flight", u);
        report(nm, (double)half, ms);
        switch (u) {
            case 1: ms = T.med_ms([&] { write1<1><<<wgs, TPB>>>(dst); }, reps); break;
            case 2: ms = T.med_ms([&] { write1<2><<<wgs, TPB>>>(dst); }, reps); break;
            case 4: ms = T.med_ms([&] { write1<4><<<wgs, TPB>>>(dst); }, reps); break;
            default: ms = T.med_ms([&] { write1<8><<<wgs, TPB>>>(dst); }, reps); break;
        }
        snprintf(nm, sizeof nm, "write-only x%d per lane", u);
        report(nm, (double)half, ms);
        switch (u) {
            case 1: ms = T.med_ms([&] { copy1<1><<<wgs, TPB>>>(src, dst); }, reps); break;
            case 2: ms = T.med_ms([&] { copy1<2><<<wgs, TPB>>>(src, dst); }, reps); break;
            case 4: ms = T.med_ms([&] { copy1<4><<<wgs, TPB>>>(src, dst); }, reps); break;
            default: ms = T.med_ms([&] { copy1<8><<<wgs, TPB>>>(src, dst); }, reps); break;
        }
        snprintf(nm, sizeof nm, "copy 1->1 x%d in flight", u);
        report(nm, 2.0 * (double)half, ms);
    }
    const long long B16 = B / 16;
    const int wps = (int)(B16 / TPB);
    struct Lay { const char* name; long long pad; bool inter; };
    const Lay lays[] = {{"dense", 0, false}, {"pad 256 B", 256, false}, {"pad 2 KiB", 2048, false},
                        {"pad 4 KiB", 4096, false}, {"pad 6 KiB", 6144, false}, {"pad 36 KiB", 36864, false},
                        {"pad 68 KiB", 69632, false}, {"chunk-interleaved 2 KiB", 0, true}};
    for (const Lay& L : lays) {
        const long long bp = L.inter ? TPB : B16 + L.pad / 16;
        const long long cp = L.inter ? (K + M) * TPB : TPB;
        const long long sp = L.inter ? (K + M) * B16 : (K + M) * bp;
        const long long S1 = std::min(S, total / 16 / sp);
        char nm[96];
        float ms = T.med_ms([&] { xor_km<10, 4><<<S1 * wps, TPB>>>(buf, sp, bp, cp, wps); }, reps);
        snprintf(nm, sizeof nm, "xor 10r->4w %s", L.name);
        report(nm, (double)S1 * 14 * B, ms);
        const long long S2 = (S1 * 14 / 11) & ~7LL;
        const long long bp2 = L.inter ? TPB : bp, cp2 = L.inter ? 11 * TPB : TPB, sp2 = L.inter ? 11 * B16 : 11 * bp;
        ms = T.med_ms([&] { xor_km<10, 1><<<S2 * wps, TPB>>>(buf, sp2, bp2, cp2, wps); }, reps);
        snprintf(nm, sizeof nm, "xor 10r->1w %s", L.name);
        report(nm, (double)S2 * 11 * B, ms);
    }
    {
        const long long bp = B16, sp = 14 * B16, sp2 = 11 * B16;
        const int wps1 = (int)(B16 / 64);
        const long long S2 = (S * 14 / 11) & ~7LL;
        float ms;
        ms = T.med_ms([&] { xor_split<10, 4, 2><<<S * wps1, 128>>>(buf, sp, bp, wps1); }, reps);
        report("split W=2 xor 10r->4w dense", (double)S * 14 * B, ms);
        ms = T.med_ms([&] { xor_split<10, 4, 4><<<S * wps1, 256>>>(buf, sp, bp, wps1); }, reps);
        report("split W=4 xor 10r->4w dense", (double)S * 14 * B, ms);
        ms = T.med_ms([&] { xor_split<10, 4, 5><<<S * wps1, 320>>>(buf, sp, bp, wps1); }, reps);
        report("split W=5 xor 10r->4w dense", (double)S * 14 * B, ms);
        ms = T.med_ms([&] { xor_split<10, 4, 1><<<S * wps1, 64>>>(buf, sp, bp, wps1); }, reps);
        report("split W=1 xor 10r->4w dense", (double)S * 14 * B, ms);
        ms = T.med_ms([&] { xor_split<10, 1, 2><<<S2 * wps1, 128>>>(buf, sp2, bp, wps1); }, reps);
        report("split W=2 xor 10r->1w dense", (double)S2 * 11 * B, ms);
        ms = T.med_ms([&] { xor_split<10, 1, 5><<<S2 * wps1, 320>>>(buf, sp2, bp, wps1); }, reps);
        report("split W=5 xor 10r->1w dense", (double)S2 * 11 * B, ms);
        ms = T.med_ms([&] { xor_split<10, 1, 10><<<S2 * wps1, 640>>>(buf, sp2, bp, wps1); }, reps);
        report("split W=10 xor 10r->1w dense", (double)S2 * 11 * B, ms);
        ms = T.med_ms([&] { xor_split<10, 4, 10><<<S * wps1, 640>>>(buf, sp, bp, wps1); }, reps);
        report("split W=10 xor 10r->4w dense", (double)S * 14 * B, ms);
    }
    {
        // ratio experiments: regions A (reads) and B (writes) inside the 56 GiB buffer
        const long long units = (S * 10 * B) / (10 * TPB * 16);  // 40 GiB of reads
        const u32x4* A = buf;
        u32x4* Bw = buf + units * 10 * TPB;
        float ms = T.med_ms([&] { rw_ratio<10, 4><<<units, TPB>>>(A, Bw); }, reps);
        report("two streams read:write 10:4", (double)units * 14 * TPB * 16, ms);
        ms = T.med_ms([&] { rw_ratio<10, 1><<<units, TPB>>>(A, Bw); }, reps);
        report("two streams read:write 10:1", (double)units * 11 * TPB * 16, ms);
        ms = T.med_ms([&] { rw_ratio<10, 0><<<units, TPB>>>(A, Bw); }, reps);
        report("one stream read 10 x 2 KiB per WG", (double)units * 10 * TPB * 16, ms);
        ms = T.med_ms([&] { rw_ratio<1, 1><<<units, TPB>>>(A, Bw); }, reps);
        report("two streams read:write 1:1", (double)units * 2 * TPB * 16, ms);
        const long long B16 = B / 16;
        const int wps = (int)(B16 / TPB);
        ms = T.med_ms([&] { stripe_read_only<10, 4><<<S * wps, TPB>>>(buf, sink, B16, wps); }, reps);
        report("stripes read-only 10 streams", (double)S * 10 * B, ms);
    }
    }  // !only_new
    {
        const long long B16 = B / 16;
        const int wps = (int)(B16 / TPB);
        const long long jobs = S * wps;
        for (int G : {2048, 4096}) {
            auto run = [&](auto kern, int J) {
                const long long per = (long long)G * J;
                for (long long j0 = 0; j0 < jobs; j0 += per) {
                    const long long n = std::min(per, jobs - j0);
                    kern<<<(unsigned)(n / J), TPB>>>(buf, B16, wps, j0);
                }
            };
            char nm[96];
            float ms;
            ms = T.med_ms([&] { run(phased_10_4<1>, 1); }, reps);
            snprintf(nm, sizeof nm, "phased G=%d J=1", G);
            report(nm, (double)S * 14 * B, ms);
            ms = T.med_ms([&] { run(phased_10_4<4>, 4); }, reps);
            snprintf(nm, sizeof nm, "phased G=%d J=4", G);
            report(nm, (double)S * 14 * B, ms);
            ms = T.med_ms([&] { run(phased_10_4<8>, 8); }, reps);
            snprintf(nm, sizeof nm, "phased G=%d J=8", G);
            report(nm, (double)S * 14 * B, ms);
            ms = T.med_ms([&] { run(phased_10_4<16>, 16); }, reps);
            snprintf(nm, sizeof nm, "phased G=%d J=16", G);
            report(nm, (double)S * 14 * B, ms);
        }
    }
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
