// Per-call rate of the device tier (tuning tool): the reference's proxy makes ONE ErasureCode call per
// stripe (proxy.cpp:312-349); with HBM-resident blocks each such call is one asynchronous launch.  This
// measures how many per-stripe calls per second the C ABI sustains (host issue cost) and the resulting
// data rate, against one batched launch over the same stripes.
// Build: hipcc -O2 -std=c++20 --offload-arch=gfx950 -Iinclude tools/call_rate.cpp -Lerasure-codes-prototype_amd/lib -lecg
//        -Wl,-rpath,'$ORIGIN/../erasure-codes-prototype_amd/lib' -o tools/call_rate
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <tuple>
#include <cstdio>
#include <cstdlib>
#include <string>
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
#define OK(x)                                                                            \
    do {                                                                                 \
        int r_ = (x);                                                                    \
        if (r_ != 0) {                                                                   \
            fprintf(stderr, "%s:%d rc=%d %s\n", __FILE__, __LINE__, r_, ecg_last_error()); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    // CALL_RATE_SCHED=spin|yield|block: the application's hipSetDeviceFlags scheduling policy, which
    // decides how hipStreamSynchronize waits (the host tier's per-call completion wait)
    if (const char* sch = getenv("CALL_RATE_SCHED")) {
        const std::string v(sch);
        const unsigned f = v == "spin" ? hipDeviceScheduleSpin : v == "yield" ? hipDeviceScheduleYield
                                                                               : hipDeviceScheduleBlockingSync;
        CK(hipSetDeviceFlags(f));
        printf("scheduling policy: %s\n", sch);
    }
    const int k = 10, m = 4, n = k + m;
    const bool host_latency_only = argc > 2 && std::string(argv[2]) == "latency";
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    int* M = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (long long B : {64LL << 10, 256LL << 10, 1LL << 20, 4LL << 20}) {
        if (host_latency_only) break;
        const int S = (int)std::min(4096LL, (16LL << 30) / (n * B));
        uint8_t* buf;
        CK(hipMalloc(&buf, (size_t)S * n * B));
        OK(ecg_fill_random(buf, (long long)S * n * B, 1, 0, st));
        std::vector<char*> ptrs((size_t)S * n);
        for (int s = 0; s < S; s++)
            for (int b = 0; b < n; b++) ptrs[(size_t)s * n + b] = (char*)(buf + ((size_t)s * n + b) * B);
        ecg_coding_parameters cp{};
        cp.k = k;
        cp.m = m;
        ecg_ec* ec = ecg_ec_factory(ECG_RS, &cp);
        OK(ecg_ec_set_memory(ec, ECG_MEM_DEVICE, st));
        for (int mode = 0; mode < 4; mode++) {
            double best_host = 1e30;
            float best_dev = 1e30f;
            for (int r = 0; r < reps + 1; r++) {
                CK(hipStreamSynchronize(st));
                CK(hipEventRecord(e0, st));
                const double t0 = now();
                if (mode == 0) {
                    for (int s = 0; s < S; s++)
                        OK(ecg_dev_matrix_encode(k, m, M, &ptrs[(size_t)s * n], &ptrs[(size_t)s * n + k], B, st));
                } else if (mode == 1) {
                    for (int s = 0; s < S; s++)
                        OK(ecg_ec_encode(ec, &ptrs[(size_t)s * n], &ptrs[(size_t)s * n + k], (int)B));
                } else if (mode == 2) {
                    OK(ecg_encode_batch(k, m, M, buf, n * B, B, buf + k * B, n * B, B, B, S, st));
                } else {  // the per-stripe loop inside a deferred-batch scope
                    OK(ecg_batch_begin());
                    for (int s = 0; s < S; s++)
                        OK(ecg_ec_encode(ec, &ptrs[(size_t)s * n], &ptrs[(size_t)s * n + k], (int)B));
                    OK(ecg_batch_end());
                }
                const double t1 = now();
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r > 0) {
                    best_host = std::min(best_host, t1 - t0);
                    best_dev = std::min(best_dev, ms);
                }
            }
            const char* names[4] = {"ecg_dev_matrix_encode per stripe", "ecg_ec_encode (device) per stripe",
                                    "ecg_encode_batch (one launch)", "ecg_ec_encode per stripe, batch scope"};
            const char* name = names[mode];
            const double data = (double)S * k * B;
            printf("B=%7lld S=%5d %-36s host %7.2f us/call  device %8.3f ms  %7.1f GiB/s data  (%5.1f%% of HBM peak)\n", B, S,
                   name, best_host / (mode == 2 ? 1 : S) * 1e6, best_dev, data / (best_dev * 1e-3) / (1 << 30),
                   (double)S * n * B / (best_dev * 1e-3) / 8e12 * 100);
            fflush(stdout);
        }
        ecg_ec_destroy(ec);
        CK(hipFree(buf));
    }
    if (argc > 2 && std::string(argv[2]) == "device") {  // device tier only (e.g. under rocprofv3)
        ecg_free(M);
        return 0;
    }

    // Host tier (synchronous calls on host buffers, the proxy's own buffers): latency per call from C++.
    for (auto [kk, mm, B] : {std::tuple<int, int, int>{6, 4, 1024}, {10, 4, 1024}, {10, 4, 16384}, {10, 4, 65536},
                             {10, 4, 1 << 20}, {10, 4, 4 << 20}}) {
        int* Mh = ecg_reed_sol_vandermonde_coding_matrix(kk, mm, 8);
        // the proxy's SET buffers (proxy.cpp:335-339): data = slices of one value buffer, parities separate
        std::vector<char> value((size_t)kk * B, 1);
        std::vector<std::vector<char>> blocks(mm, std::vector<char>(B, 1));
        std::vector<char*> p(kk + mm);
        for (int i = 0; i < kk; i++) p[i] = value.data() + (size_t)i * B;
        for (int i = 0; i < mm; i++) p[kk + i] = blocks[i].data();
        const int calls = B >= (1 << 20) ? 100 : 4000;
        OK(ecg_jerasure_matrix_encode(kk, mm, 8, Mh, p.data(), p.data() + kk, B));
        double t0 = now();
        for (int c = 0; c < calls; c++) OK(ecg_jerasure_matrix_encode(kk, mm, 8, Mh, p.data(), p.data() + kk, B));
        const double enc = (now() - t0) / calls * 1e6;
        int er[2] = {2, -1};
        t0 = now();
        for (int c = 0; c < calls; c++) OK(ecg_jerasure_matrix_decode(kk, mm, 8, Mh, 1, er, p.data(), p.data() + kk, B));
        const double dec = (now() - t0) / calls * 1e6;
        printf("host tier RS(%d,%d) B=%6d  encode %6.1f us/call  decode %6.1f us/call\n", kk, mm, B, enc, dec);
        fflush(stdout);
        ecg_free(Mh);
    }
    if (host_latency_only) {
        ecg_free(M);
        return 0;
    }
    // Concurrent host-tier callers (the proxy runs encode on detached threads, proxy.cpp:416-419):
    // T threads, each with its own buffers, issuing synchronous RS(6,4) / RS(10,4) calls.
    for (auto [kk, mm, B] : {std::tuple<int, int, int>{6, 4, 1024}, {10, 4, 65536}, {10, 4, 1 << 20}}) {
        int* Mh = ecg_reed_sol_vandermonde_coding_matrix(kk, mm, 8);
        for (int T : {1, 2, 4, 8, 16}) {
            const int calls = B >= (1 << 20) ? 100 : 2000;
            std::vector<std::thread> th;
            std::atomic<int> errors{0};
            const double t0 = now();
            for (int t = 0; t < T; t++)
                th.emplace_back([&, t] {
                    std::vector<std::vector<char>> blocks(kk + mm, std::vector<char>(B, (char)t));
                    std::vector<char*> p(kk + mm);
                    for (int i = 0; i < kk + mm; i++) p[i] = blocks[i].data();
                    for (int c = 0; c < calls; c++)
                        if (ecg_jerasure_matrix_encode(kk, mm, 8, Mh, p.data(), p.data() + kk, B) != 0) errors++;
                });
            for (auto& x : th) x.join();
            const double dt = now() - t0;
            printf("host tier RS(%d,%d) B=%7d  %2d threads: %8.0f calls/s  (%.1f us/call/thread, %.1f GB/s over PCIe)%s\n",
                   kk, mm, B, T, T * calls / dt, dt / calls * 1e6, (double)T * calls * (kk + mm) * B / dt / 1e9,
                   errors ? "  ERRORS" : "");
            fflush(stdout);
        }
        ecg_free(Mh);
    }
    // Thread per request (the proxy starts a detached thread per SET and encodes on it, proxy.cpp:416-419):
    // each request is a new thread making ONE host-tier call.  Reported with the bare thread start/join
    // cost alongside, so the difference is what the library adds to a cold thread's first call.
    for (auto [kk, mm, B] : {std::tuple<int, int, int>{6, 4, 1024}, {10, 4, 65536}, {10, 4, 1 << 20}}) {
        int* Mh = ecg_reed_sol_vandermonde_coding_matrix(kk, mm, 8);
        std::vector<std::vector<char>> blocks(kk + mm, std::vector<char>(B, 3));
        std::vector<char*> p(kk + mm);
        for (int i = 0; i < kk + mm; i++) p[i] = blocks[i].data();
        const int reqs = B >= (1 << 20) ? 100 : 500;
        std::atomic<int> errors{0};
        double t0 = now();
        for (int r = 0; r < reqs; r++) std::thread([] {}).join();
        const double bare = (now() - t0) / reqs * 1e6;
        t0 = now();
        for (int r = 0; r < reqs; r++)
            std::thread([&] {
                if (ecg_jerasure_matrix_encode(kk, mm, 8, Mh, p.data(), p.data() + kk, B) != 0) errors++;
            }).join();
        const double per = (now() - t0) / reqs * 1e6;
        printf("thread per request RS(%d,%d) B=%7d: %7.1f us/request (bare thread %.1f us)%s\n", kk, mm, B, per, bare,
               errors ? "  ERRORS" : "");
        fflush(stdout);
        ecg_free(Mh);
    }
    ecg_free(M);
    return 0;
}
