// Back-to-back launch floor on one stream (tuning probe, not shipped): what one in-order kernel costs the
// GPU timeline when its work is tiny, as a function of the kernel-argument size.  The device tier's
// per-call path (one ErasureCode call per stripe on HBM blocks) is one such launch per call, with a
// ~1.4 KiB GfLaunch argument block (160 inline block pointers).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 profiles/r04/lat_tables/launch_floor.hip -o profiles/r04/lat_tables/launch_floor
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <int N>
struct Args {
    unsigned* out;
    const unsigned* in;
    long long n;
    unsigned char pad[N];
};

template <int N>
__global__ void copy_kernel(const Args<N> a) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) a.out[i] = a.in[i] ^ a.pad[0];
}

static double g_host_us;  // host time per launch of the last run()

template <int N>
float run(int launches, long long bytes, unsigned* out, const unsigned* in, hipStream_t st, hipEvent_t e0,
          hipEvent_t e1, unsigned flags) {
    Args<N> a;
    a.out = out;
    a.in = in;
    a.n = bytes / 4;
    for (int i = 0; i < N; i++) a.pad[i] = 0;
    const int threads = 256;
    const unsigned blocks = (unsigned)((a.n + threads - 1) / threads);
    float best = 1e30f;
    double best_host = 1e30;
    for (int r = 0; r < 4; r++) {
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        const auto h0 = std::chrono::steady_clock::now();
        for (int i = 0; i < launches; i++) {
            void* argv[] = {(void*)&a};
            if (flags) CK(hipExtLaunchKernel((const void*)copy_kernel<N>, dim3(blocks), dim3(threads), argv, 0, st,
                                             nullptr, nullptr, flags));
            else CK(hipLaunchKernel((const void*)copy_kernel<N>, dim3(blocks), dim3(threads), argv, 0, st));
        }
        const double host = std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
        if (r > 0 && host < best_host) best_host = host;
    }
    g_host_us = best_host * 1e6 / launches;
    return best * 1000.f / launches;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    unsigned *in, *out;
    CK(hipMalloc(&in, 4 << 20));
    CK(hipMalloc(&out, 4 << 20));
    CK(hipMemset(in, 1, 4 << 20));
    const int L = 4000;
    for (long long bytes : {4LL, 4096LL, 65536LL, 1LL << 20}) {
        float dv[4];
        double hv[4];
        dv[0] = run<1>(L, bytes, out, in, st, e0, e1, 0);
        hv[0] = g_host_us;
        dv[1] = run<256>(L, bytes, out, in, st, e0, e1, 0);
        hv[1] = g_host_us;
        dv[2] = run<1408>(L, bytes, out, in, st, e0, e1, 0);
        hv[2] = g_host_us;
        dv[3] = run<4072>(L, bytes, out, in, st, e0, e1, 0);
        hv[3] = g_host_us;
        printf("copy %8lld B, device (host) us per launch: args 24 B %5.2f (%5.2f) | 280 B %5.2f (%5.2f) | "
               "1432 B %5.2f (%5.2f) | 4096 B %5.2f (%5.2f)\n",
               bytes, dv[0], hv[0], dv[1], hv[1], dv[2], hv[2], dv[3], hv[3]);
        fflush(stdout);
    }
    // hipExtAnyOrderLaunch: no barrier bit on the packet, so independent launches on one stream may overlap
    for (long long bytes : {4LL, 65536LL, 1LL << 20}) {
        printf("any-order copy %8lld B: args 24 B %6.2f us | 1432 B %6.2f us per launch\n", bytes,
               run<1>(L, bytes, out, in, st, e0, e1, 1), run<1408>(L, bytes, out, in, st, e0, e1, 1));
        fflush(stdout);
    }
    return 0;
}
