// Cache-policy bits of the streaming loads and stores on the encode's access pattern (tuning tool, not
// shipped).  The engine streams with __builtin_nontemporal_load / _store (global_load/store_dwordx4 ... nt).
// gfx950's vector memory instructions also carry the scope bits sc0 / sc1, which decide how far down the
// cache hierarchy an access is kept coherent (and, for stores, written through).  This times the stripe
// pattern of tools/hbm_ceiling.hip's xor_km<10,4> (10 read streams -> 4 written, [S][14][1 MiB], XCD-contiguous
// map, no GF multiply) with every load policy x store policy below, on two separate 56 GiB buffers
// (placement sets 0.77 vs 0.79 per buffer, profiles/r03/placement/), interleaved over rounds.
//   load  0: nt   1: nt sc1   2: nt sc0 sc1   3: sc1   4: plain
//   store 0: nt   1: nt sc1   2: nt sc0 sc1   3: sc0 sc1   4: plain
// as raw buffer loads / stores (the policy is an operand of the compiler builtin), plus the engine's own
// global_load / global_store ... nt form for reference.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/policy_probe tools/policy_probe.hip
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
constexpr int K = 10, M = 4;

// Buffer loads / stores with the policy in the instruction's cache-policy field (compiler builtins, so
// the compiler tracks the outstanding accesses): nt = 2, sc0 = 1, sc1 = 16.  Each workgroup's resource
// covers its own stripe (14 MiB): an offset outside it reads 0 and drops the write, never faults.
constexpr int kBufWord3 = 0x00020000;  // gfx9 raw-buffer descriptor word 3 (32-bit data format)

__device__ __forceinline__ long long xcd_map(long long b) {
    const long long per = (long long)gridDim.x >> 3;
    return (b & 7) * per + (b >> 3);
}

template <int LAUX, int SAUX>  // cache-policy operands (immediates)
__global__ void __launch_bounds__(TPB) xor_10_4(u32x4* __restrict__ base, long long sp16, long long bp16, int wg_per_stripe) {
    const long long w = xcd_map(blockIdx.x);
    const long long s = w / wg_per_stripe;
    const long long ch = w - s * wg_per_stripe;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(base + s * sp16, 0, (int)((K + M) * bp16 * 16), kBufWord3);
    const int o0 = (int)((ch * TPB + threadIdx.x) * 16);
    const int bstep = (int)(bp16 * 16);
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, o0 + j * bstep, 0, LAUX);
    u32x4 a = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= x[j];
#pragma unroll
    for (int p = 0; p < M; ++p) {
        u32x4 o = a;
        o.x ^= p;
        __builtin_amdgcn_raw_buffer_store_b128(o, r, o0 + (K + p) * bstep, 0, SAUX);
    }
}

// the engine's form: global_load / global_store ... nt through the compiler's non-temporal builtins
__global__ void __launch_bounds__(TPB) xor_10_4_global(u32x4* __restrict__ base, long long sp16, long long bp16,
                                                       int wg_per_stripe) {
    const long long w = xcd_map(blockIdx.x);
    const long long s = w / wg_per_stripe;
    const long long ch = w - s * wg_per_stripe;
    u32x4* sp = base + s * sp16 + ch * TPB + threadIdx.x;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = __builtin_nontemporal_load(sp + j * bp16);
    u32x4 a = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= x[j];
#pragma unroll
    for (int p = 0; p < M; ++p) {
        u32x4 o = a;
        o.x ^= p;
        __builtin_nontemporal_store(o, sp + (K + p) * bp16);
    }
}

typedef void (*Kern)(u32x4*, long long, long long, int);

struct Variant {
    const char* name;
    Kern k;
};

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    const long long B = 1 << 20, S = 4096;
    const long long bytes = S * (K + M) * B;
    const long long B16 = B / 16, sp16 = (K + M) * B16;
    const int wg_per_stripe = (int)(B16 / TPB);
    const long long grid = S * wg_per_stripe;
    std::vector<Variant> vs = {
        {"global ld nt / st nt (engine)", xor_10_4_global},
        {"buffer ld nt / st nt          ", xor_10_4<2, 2>}, {"buffer ld nt / st nt sc1      ", xor_10_4<2, 18>},
        {"buffer ld nt / st nt sc0 sc1  ", xor_10_4<2, 19>}, {"buffer ld nt / st sc0 sc1     ", xor_10_4<2, 17>},
        {"buffer ld nt / st plain       ", xor_10_4<2, 0>}, {"buffer ld nt sc1 / st nt      ", xor_10_4<18, 2>},
        {"buffer ld nt sc0 sc1 / st nt  ", xor_10_4<19, 2>}, {"buffer ld sc1 / st nt         ", xor_10_4<16, 2>},
        {"buffer ld plain / st nt       ", xor_10_4<0, 2>}, {"buffer ld nt sc1 / st nt sc1  ", xor_10_4<18, 18>},
    };
    u32x4* buf[2];
    for (auto& b : buf) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 0x5a, bytes));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size() * 2);
    for (int r = -1; r < rounds; ++r) {  // round -1: warm-up
        for (int bi = 0; bi < 2; ++bi) {
            for (size_t v = 0; v < vs.size(); ++v) {
                for (int i = 0; i < reps; ++i) {
                    CK(hipEventRecord(e0));
                    hipLaunchKernelGGL(vs[v].k, dim3((unsigned)grid), dim3(TPB), 0, 0, buf[bi], sp16, B16, wg_per_stripe);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (r >= 0) t[v * 2 + bi].push_back(ms);
                }
            }
        }
    }
    printf("stripes [%lld][14][1 MiB], 10 -> 4 XOR, XCD-contiguous map; fraction of 8 TB/s, median per buffer\n", S);
    for (size_t v = 0; v < vs.size(); ++v) {
        printf("%s", vs[v].name);
        for (int bi = 0; bi < 2; ++bi) {
            auto x = t[v * 2 + bi];
            std::sort(x.begin(), x.end());
            const double med = x[x.size() / 2];
            printf("   buf%d %.4f", bi, (double)bytes / (med * 1e-3) / 8e12);
        }
        printf("\n");
    }
    for (auto& b : buf) CK(hipFree(b));
    return 0;
}
