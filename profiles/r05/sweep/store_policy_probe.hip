// Store cache policy of the encode's access path (round 5 probe; not shipped).
//
// The encode's movement: S = 4096 stripes of [14][1 MiB] blocks, 128-thread workgroups each taking a 2 KiB
// chunk of every block, XCD-contiguous grid map (gf_vec_kernel, grid map 1), non-temporal 16-byte loads of
// the 10 data blocks, 4 parity blocks written.  Here the parity is a XOR (BINARY, every mask ~0), and the
// store instruction's cache policy varies:
//   SP 0  plain                     (line kept in the XCD's L2, written back on eviction)
//   SP 1  nt       (the product)    (line kept in L2; MI355X_MICROARCH.md "stores of each flavour")
//   SP 2  sc1                       (line dropped from L2: write-through)
//   SP 3  sc0 sc1                   (dropped)
//   SP 4  sc1 nt
// Policies 2-4 are vector stores written with inline asm (global_store_dwordx4 with cache-policy bits).
// Every variant's parities are checked on the host for a few stripes; fractions = (10 + 4) * B * S / time / 8 TB/s,
// HIP events, variants interleaved round by round.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 profiles/r05/sweep/store_policy_probe.hip -o tools/store_policy_probe
// Run:   tools/store_policy_probe [rounds=4] [reps=10] [stripes=4096]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kK = 10, kM = 4, kN = 14, kThreads = 128;

template <int SP>
__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) {
    if constexpr (SP == 0) *reinterpret_cast<u32x4*>(p) = v;
    else if constexpr (SP == 1) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
}

// parity of a 16-byte column = XOR of the 10 inputs, with the constant {1, 2, 3, 4} folded into dwords 0-3
template <int SP>
__global__ void __launch_bounds__(kThreads, 6) encode_xor(uint8_t* base, long long B, int wg_per_stripe) {
    long long b = blockIdx.x;
    const long long per = (long long)gridDim.x >> 3;  // grid % 8 == 0 (host)
    b = (b & 7) * per + (b >> 3);
    const long long s = b / wg_per_stripe, w = b - s * wg_per_stripe;
    uint8_t* st = base + s * kN * B;
    const long long off = (w * kThreads + threadIdx.x) << 4;
    if (off >= B) return;
    u32x4 acc[kM];
#pragma unroll
    for (int p = 0; p < kM; p++) acc[p] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int j0 = 0; j0 < kK; j0 += 5) {
        u32x4 x[5];
#pragma unroll
        for (int u = 0; u < 5; u++) x[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(st + (j0 + u) * B + off));
#pragma unroll
        for (int u = 0; u < 5; u++)
#pragma unroll
            for (int p = 0; p < kM; p++) acc[p] ^= (j0 + u == p) ? (x[u] ^ u32x4{1u, 2u, 3u, 4u}) : x[u];
    }
#pragma unroll
    for (int p = 0; p < kM; p++) store16<SP>(st + (kK + p) * B + off, acc[p]);
}

using Kern = void (*)(uint8_t*, long long, int);

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 4, reps = argc > 2 ? atoi(argv[2]) : 10;
    const int S = argc > 3 ? atoi(argv[3]) : 4096;
    const long long B = 1 << 20;
    uint8_t* d = nullptr;
    const size_t bytes = (size_t)S * kN * B;
    CK(hipMalloc(&d, bytes));
    {
        std::vector<uint8_t> h((size_t)kN * B);
        for (size_t i = 0; i < h.size(); i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
        for (int s = 0; s < S; s++) CK(hipMemcpy(d + (size_t)s * kN * B, h.data(), h.size(), hipMemcpyHostToDevice));
    }
    const int wps = (int)(B / 16 / kThreads);
    const unsigned grid = (unsigned)((long long)S * wps);
    if (grid % 8) return 1;
    struct V {
        const char* name;
        Kern k;
        std::vector<double> ms;
    };
    std::vector<V> vs = {{"plain", encode_xor<0>, {}}, {"nt (product)", encode_xor<1>, {}}, {"sc1", encode_xor<2>, {}},
                         {"sc0 sc1", encode_xor<3>, {}}, {"sc1 nt", encode_xor<4>, {}}};
    std::vector<hipEvent_t> ev(reps + 1);
    for (auto& e : ev) CK(hipEventCreate(&e));
    for (V& v : vs) {  // every variant writes the same parities: check each once, from zeroed parity blocks
        for (int s : {0, S / 2 + 1, S - 1}) CK(hipMemset(d + ((size_t)s * kN + kK) * B, 0, (size_t)kM * B));
        hipLaunchKernelGGL(v.k, dim3(grid), dim3(kThreads), 0, nullptr, d, B, wps);
        CK(hipDeviceSynchronize());
        for (int s : {0, S / 2 + 1, S - 1}) {
            std::vector<uint8_t> h((size_t)kN * B);
            CK(hipMemcpy(h.data(), d + (size_t)s * kN * B, h.size(), hipMemcpyDeviceToHost));
            for (int p = 0; p < kM; p++)
                for (long long x = 0; x < B; x += 4093) {
                    uint8_t want = 0;
                    for (int j = 0; j < kK; j++) want ^= h[(size_t)j * B + x];
                    if (p < kK) want ^= (uint8_t)(((x & 15) >> 2) + 1) * (((x & 3) == 0) ? 1 : 0);
                    if (h[(size_t)(kK + p) * B + x] != want) {
                        fprintf(stderr, "%s: parity %d of stripe %d wrong at %lld\n", v.name, p, s, x);
                        return 2;
                    }
                }
        }
    }
    for (int r = 0; r < rounds; r++)
        for (V& v : vs) {
            for (int w = 0; w < 2; w++) hipLaunchKernelGGL(v.k, dim3(grid), dim3(kThreads), 0, nullptr, d, B, wps);
            CK(hipEventRecord(ev[0], nullptr));
            for (int i = 0; i < reps; i++) {
                hipLaunchKernelGGL(v.k, dim3(grid), dim3(kThreads), 0, nullptr, d, B, wps);
                CK(hipEventRecord(ev[i + 1], nullptr));
            }
            CK(hipEventSynchronize(ev[reps]));
            for (int i = 0; i < reps; i++) {
                float ms = 0;
                CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
                v.ms.push_back(ms);
            }
        }
    const double alg = (double)S * kN * B;
    for (V& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        double avg = 0;
        for (double x : v.ms) avg += x;
        avg /= v.ms.size();
        printf("store %-14s avg %.4f ms  median %.4f  | frac avg %.4f  median %.4f\n", v.name, avg, v.ms[v.ms.size() / 2],
               alg / (avg * 1e-3) / 8e12, alg / (v.ms[v.ms.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
