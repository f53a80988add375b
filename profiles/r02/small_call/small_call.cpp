// Where the time of one small synchronous host-tier call goes (config 1's shape: RS(6,4), 1 KiB blocks,
// one jerasure_matrix_encode per stripe on the proxy's host buffers, proxy.cpp:312-349).
//   call     ecg_jerasure_matrix_encode, RS(6,4) 1 KiB (the product path: gather into pinned mapped
//            staging, one zero-copy kernel over PCIe, synchronize, scatter back)
//   empty    an empty kernel + hipStreamSynchronize on a non-blocking stream: the launch + completion
//            round trip every synchronous GPU call pays, whatever it computes
//   touch    a kernel that reads 6 KiB and writes 4 KiB of pinned mapped host memory (one 16-byte load per
//            lane per block, like the product kernel) + synchronize: empty + the PCIe traffic
//   par      the same with all six loads issued before the first use (one PCIe round trip)
//   read1    one 1 KiB block read, four written;   write   four written, nothing read
//   emptyF / parF   empty / par, completing by a flag the kernel posts in mapped host memory (host polls)
//   parFbig  parF with the product's ~1.5 KiB kernel-argument block (no measurable cost)
//   parFtab  parF plus 24 coefficient words read through scalar loads from a device table (no cost
//            when the loads are not behind per-input branches)
//   parFcp   parF plus the call's host-side gather (6 KiB) and scatter (4 KiB) memcpys: the floor of a
//            zero-copy call
//   callD / call16, decD / dec16   the product's encode / decode with the latency kernel at 4 bytes
//            per lane (ECG_OPT_LAT_DWORD_BYTES default) and at 16 bytes per lane (option 0), alternated
// Run under rocprofv3 --kernel-trace --hip-trace --stats to split each into API and kernel time.
// Build: hipcc -O2 -std=c++20 --offload-arch=gfx950 -Iinclude profiles/r02/small_call/small_call.cpp -Lerasure-codes-prototype_amd/lib -lecg
//        -Wl,-rpath,'$ORIGIN/../erasure-codes-prototype_amd/lib' -o profiles/r02/small_call/small_call
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ecg.h"

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void empty_kernel() {}

// 64 lanes x 16 B = 1 KiB per block: each lane loads its 16 bytes of k input blocks and stores m outputs
__global__ void touch_kernel(const uint4* in, uint4* out, int k, int m) {
    const int lane = threadIdx.x;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < k; j++) {
        const uint4 v = in[j * 64 + lane];
        acc.x ^= v.x;
        acc.y ^= v.y;
        acc.z ^= v.z;
        acc.w ^= v.w;
    }
    for (int p = 0; p < m; p++) out[p * 64 + lane] = acc;
}

// the same traffic with every load issued before the first use (compile-time K, M): one PCIe round trip
template <int K, int M>
__global__ void touch_parallel_kernel(const uint4* in, uint4* out) {
    const int lane = threadIdx.x;
    uint4 v[K];
#pragma unroll
    for (int j = 0; j < K; j++) v[j] = in[j * 64 + lane];
    uint4 acc = v[0];
#pragma unroll
    for (int j = 1; j < K; j++) {
        acc.x ^= v[j].x;
        acc.y ^= v[j].y;
        acc.z ^= v[j].z;
        acc.w ^= v[j].w;
    }
#pragma unroll
    for (int p = 0; p < M; p++) out[p * 64 + lane] = acc;
}

// writes only (posted PCIe writes), no host reads
__global__ void write_only_kernel(uint4* out, int m) {
    const int lane = threadIdx.x;
    for (int p = 0; p < m; p++) out[p * 64 + lane] = make_uint4(lane, p, 0, 0);
}

// completion flag in mapped host memory: after the wave's stores, lane 0 publishes `seq` with a
// system-scope release (a vector store); the host spins on the flag instead of synchronizing the stream
__device__ __forceinline__ void publish(unsigned* flag, unsigned seq) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void empty_flag_kernel(unsigned* flag, unsigned seq) { publish(flag, seq); }

template <int K, int M>
__global__ void touch_parallel_flag_kernel(const uint4* in, uint4* out, unsigned* flag, unsigned seq) {
    const int lane = threadIdx.x;
    uint4 v[K];
#pragma unroll
    for (int j = 0; j < K; j++) v[j] = in[j * 64 + lane];
    uint4 acc = v[0];
#pragma unroll
    for (int j = 1; j < K; j++) {
        acc.x ^= v[j].x;
        acc.y ^= v[j].y;
        acc.z ^= v[j].z;
        acc.w ^= v[j].w;
    }
#pragma unroll
    for (int p = 0; p < M; p++) out[p * 64 + lane] = acc;
    publish(flag, seq);
}

// parF with the product's kernel-argument size: the pointers travel in a ~1.5 KiB struct (GfLaunch
// carries 128 input + 32 output inline pointers), to see what a large kernarg block costs per launch
struct BigArgs {
    const uint4* in;
    uint4* out;
    unsigned* flag;
    unsigned seq;
    const void* pad[180];
};

__global__ void touch_parallel_flag_big_kernel(const BigArgs a) {
    const int lane = threadIdx.x;
    uint4 v[6];
#pragma unroll
    for (int j = 0; j < 6; j++) v[j] = a.in[j * 64 + lane];
    uint4 acc = v[0];
#pragma unroll
    for (int j = 1; j < 6; j++) {
        acc.x ^= v[j].x;
        acc.y ^= v[j].y;
        acc.z ^= v[j].z;
        acc.w ^= v[j].w;
    }
#pragma unroll
    for (int p = 0; p < 4; p++) a.out[p * 64 + lane] = acc;
    publish(a.flag, a.seq);
}

// parF plus 24 coefficient words read from a device-memory table through scalar loads (the product
// kernel's CoefTab fetch), folded into the result so the loads cannot be dropped
__global__ void touch_parallel_flag_tab_kernel(const uint4* in, uint4* out, const __attribute__((address_space(4))) unsigned* tab,
                                               unsigned* flag, unsigned seq) {
    const int lane = threadIdx.x;
    uint4 v[6];
#pragma unroll
    for (int j = 0; j < 6; j++) v[j] = in[j * 64 + lane];
    uint4 acc = v[0];
#pragma unroll
    for (int j = 1; j < 6; j++) {
        acc.x ^= v[j].x & tab[j * 8];
        acc.y ^= v[j].y & tab[j * 8 + 1];
        acc.z ^= v[j].z & tab[j * 8 + 2];
        acc.w ^= v[j].w & tab[j * 8 + 3];
    }
#pragma unroll
    for (int p = 0; p < 4; p++) out[p * 64 + lane] = acc;
    publish(flag, seq);
}

static void spin(volatile unsigned* flag, unsigned seq, hipStream_t st) {
    const double t0 = now();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        if (now() - t0 > 1.0) {  // never wait forever on a flag: fall back to the stream
            CK(hipStreamSynchronize(st));
            if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) { fprintf(stderr, "flag never set\n"); exit(3); }
            return;
        }
    }
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4000;
    const int k = 6, m = 4, B = 1024;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint8_t *h = nullptr, *d = nullptr;
    CK(hipHostMalloc((void**)&h, (size_t)(k + m) * B, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&d, h, 0));
    for (int i = 0; i < (k + m) * B; i++) h[i] = (uint8_t)i;

    int* M = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
    std::vector<char> value((size_t)k * B, 1);
    std::vector<std::vector<char>> par(m, std::vector<char>(B, 0));
    std::vector<char*> p(k + m);
    for (int i = 0; i < k; i++) p[i] = value.data() + (size_t)i * B;
    for (int i = 0; i < m; i++) p[k + i] = par[i].data();

    auto bench = [&](const char* name, auto fn) {
        for (int i = 0; i < 200; i++) fn();  // warm
        double best = 1e9, sum = 0;
        for (int r = 0; r < 5; r++) {
            const double t0 = now();
            for (int i = 0; i < N / 5; i++) fn();
            const double us = (now() - t0) / (N / 5) * 1e6;
            best = std::min(best, us);
            sum += us;
        }
        printf("%-6s %7.2f us/call (best of 5 rounds), %7.2f avg\n", name, best, sum / 5);
        fflush(stdout);
    };
    bench("call", [&] {
        if (ecg_jerasure_matrix_encode(k, m, 8, M, p.data(), p.data() + k, B) != 0) exit(2);
    });
    bench("empty", [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
        CK(hipStreamSynchronize(st));
    });
    bench("touch", [&] {
        hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, st, (const uint4*)d, (uint4*)(d + (size_t)k * B), k, m);
        CK(hipStreamSynchronize(st));
    });
    bench("par", [&] {
        hipLaunchKernelGGL((touch_parallel_kernel<6, 4>), dim3(1), dim3(64), 0, st, (const uint4*)d, (uint4*)(d + (size_t)k * B));
        CK(hipStreamSynchronize(st));
    });
    bench("read1", [&] {
        hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, st, (const uint4*)d, (uint4*)(d + (size_t)k * B), 1, m);
        CK(hipStreamSynchronize(st));
    });
    bench("write", [&] {
        hipLaunchKernelGGL(write_only_kernel, dim3(1), dim3(64), 0, st, (uint4*)(d + (size_t)k * B), m);
        CK(hipStreamSynchronize(st));
    });
    unsigned* hflag = nullptr;
    unsigned* dflag = nullptr;
    CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
    *hflag = 0;
    unsigned seq = 0;
    bench("emptyF", [&] {
        ++seq;
        hipLaunchKernelGGL(empty_flag_kernel, dim3(1), dim3(64), 0, st, dflag, seq);
        spin(hflag, seq, st);
    });
    bench("parF", [&] {
        ++seq;
        hipLaunchKernelGGL((touch_parallel_flag_kernel<6, 4>), dim3(1), dim3(64), 0, st, (const uint4*)d,
                           (uint4*)(d + (size_t)k * B), dflag, seq);
        spin(hflag, seq, st);
    });
    bench("parF+s", [&] {  // the flag, then a stream synchronize that should find the kernel done
        ++seq;
        hipLaunchKernelGGL((touch_parallel_flag_kernel<6, 4>), dim3(1), dim3(64), 0, st, (const uint4*)d,
                           (uint4*)(d + (size_t)k * B), dflag, seq);
        spin(hflag, seq, st);
        CK(hipStreamSynchronize(st));
    });
    BigArgs big{};
    big.in = (const uint4*)d;
    big.out = (uint4*)(d + (size_t)k * B);
    big.flag = dflag;
    bench("parFbig", [&] {
        big.seq = ++seq;
        hipLaunchKernelGGL(touch_parallel_flag_big_kernel, dim3(1), dim3(64), 0, st, big);
        spin(hflag, seq, st);
    });
    unsigned* dtab = nullptr;
    CK(hipMalloc((void**)&dtab, 4096));
    CK(hipMemset(dtab, 0xff, 4096));
    CK(hipDeviceSynchronize());
    bench("parFtab", [&] {
        ++seq;
        hipLaunchKernelGGL(touch_parallel_flag_tab_kernel, dim3(1), dim3(64), 0, st, (const uint4*)d,
                           (uint4*)(d + (size_t)k * B), (const __attribute__((address_space(4))) unsigned*)dtab, dflag, seq);
        spin(hflag, seq, st);
    });
    // parF plus the call's host-side gather into staging and scatter back (6 KiB in, 4 KiB out)
    bench("parFcp", [&] {
        ++seq;
        for (int i = 0; i < k; i++) memcpy(h + (size_t)i * B, p[i], B);
        hipLaunchKernelGGL((touch_parallel_flag_kernel<6, 4>), dim3(1), dim3(64), 0, st, (const uint4*)d,
                           (uint4*)(d + (size_t)k * B), dflag, seq);
        spin(hflag, seq, st);
        for (int i = 0; i < m; i++) memcpy(p[k + i], h + (size_t)(k + i) * B, B);
    });
    // A/B of the latency kernel's lane width (ECG_OPT_LAT_DWORD_BYTES: 4 bytes per lane vs 16), alternated
    const long long lat_default = ecg_get_option(ECG_OPT_LAT_DWORD_BYTES);
    int erasures[3] = {2, -1, -1};
    for (int r = 0; r < 2; r++) {
        for (long long opt : {lat_default, 0LL}) {
            ecg_set_option(ECG_OPT_LAT_DWORD_BYTES, opt);
            bench(opt ? "callD" : "call16", [&] {
                if (ecg_jerasure_matrix_encode(k, m, 8, M, p.data(), p.data() + k, B) != 0) exit(2);
            });
            bench(opt ? "decD" : "dec16", [&] {
                if (ecg_jerasure_matrix_decode(k, m, 8, M, 1, erasures, p.data(), p.data() + k, B) != 0) exit(2);
            });
        }
    }
    ecg_set_option(ECG_OPT_LAT_DWORD_BYTES, lat_default);
    CK(hipStreamSynchronize(st));
    CK(hipFree(dtab));
    CK(hipHostFree(hflag));
    ecg_free(M);
    CK(hipHostFree(h));
    return 0;
}
