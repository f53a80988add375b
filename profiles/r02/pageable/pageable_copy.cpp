// Host->device strategies for ONE per-stripe call on pageable memory (tuning tool): the reference hands
// jerasure_matrix_encode k slices of one contiguous value buffer (proxy.cpp:337-339) and m separate
// coding buffers.  Compares, for 10 x 1 MiB in + 4 x 1 MiB out:
//   (a) per-block pageable hipMemcpyAsync (the driver stages each block),
//   (b) hipHostRegister of the caller's buffers, direct DMA, unregister,
//   (c) T host threads memcpy into pinned staging, one DMA each way.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

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

static void par_memcpy(char* dst, const char* src, size_t n, int T) {
    if (T <= 1) {
        memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n / T + 4095) & ~(size_t)4095;
    for (int t = 0; t < T; t++) {
        const size_t a = std::min(n, per * t), b = std::min(n, per * (t + 1));
        if (a < b) th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
    }
    for (auto& x : th) x.join();
}

int main() {
    const size_t B = 1 << 20;
    const int k = 10, m = 4, reps = 30;
    std::vector<char> value(k * B), coding(m * B);  // pageable, like the proxy's buffers
    for (size_t i = 0; i < value.size(); i++) value[i] = (char)i;
    char* d;
    CK(hipMalloc(&d, (k + m) * B));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    char* pin;
    CK(hipHostMalloc((void**)&pin, (k + m) * B, hipHostMallocDefault));
    auto bench = [&](const char* name, auto fn) {
        fn();
        double best = 1e30, sum = 0;
        for (int r = 0; r < reps; r++) {
            const double t0 = now();
            fn();
            const double dt = now() - t0;
            best = std::min(best, dt);
            sum += dt;
        }
        printf("%-52s best %7.1f us  mean %7.1f us  (%5.1f GB/s in+out)\n", name, best * 1e6, sum / reps * 1e6,
               (k + m) * B / best / 1e9);
        fflush(stdout);
    };
    bench("(a) per-block pageable hipMemcpyAsync", [&] {
        for (int i = 0; i < k; i++) CK(hipMemcpyAsync(d + i * B, value.data() + i * B, B, hipMemcpyHostToDevice, st));
        for (int i = 0; i < m; i++) CK(hipMemcpyAsync(coding.data() + i * B, d + (k + i) * B, B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    bench("(a') one pageable copy of the contiguous value buffer", [&] {
        CK(hipMemcpyAsync(d, value.data(), k * B, hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(coding.data(), d + k * B, m * B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    std::vector<std::vector<char>> sep(m, std::vector<char>(B));  // proxy.cpp:335: one vector per parity
    bench("(d) one H2D of the value buffer + per-block D2H (separate)", [&] {
        CK(hipMemcpyAsync(d, value.data(), k * B, hipMemcpyHostToDevice, st));
        for (int i = 0; i < m; i++) CK(hipMemcpyAsync(sep[i].data(), d + (k + i) * B, B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    bench("(e) one H2D + register each parity buffer, DMA, unregister", [&] {
        CK(hipMemcpyAsync(d, value.data(), k * B, hipMemcpyHostToDevice, st));
        for (int i = 0; i < m; i++) CK(hipHostRegister(sep[i].data(), B, hipHostRegisterDefault));
        for (int i = 0; i < m; i++) CK(hipMemcpyAsync(sep[i].data(), d + (k + i) * B, B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        for (int i = 0; i < m; i++) CK(hipHostUnregister(sep[i].data()));
    });
    bench("(f) one H2D + D2H to pinned + 1-thread memcpy out", [&] {
        CK(hipMemcpyAsync(d, value.data(), k * B, hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(pin + k * B, d + k * B, m * B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        for (int i = 0; i < m; i++) memcpy(sep[i].data(), pin + (k + i) * B, B);
    });
    bench("(g) per-block H2D (10) + per-block D2H (4), separate", [&] {
        for (int i = 0; i < k; i++) CK(hipMemcpyAsync(d + i * B, value.data() + i * B, B, hipMemcpyHostToDevice, st));
        for (int i = 0; i < m; i++) CK(hipMemcpyAsync(sep[i].data(), d + (k + i) * B, B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    hipStream_t ds[4];
    for (auto& x : ds) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipEvent_t kd;
    CK(hipEventCreateWithFlags(&kd, hipEventDisableTiming));
    for (int ns : {2, 4}) {
        char nm[96];
        snprintf(nm, sizeof nm, "(h) one H2D + per-block D2H on %d streams (separate)", ns);
        bench(nm, [&] {
            CK(hipMemcpyAsync(d, value.data(), k * B, hipMemcpyHostToDevice, st));
            CK(hipEventRecord(kd, st));
            for (int i = 0; i < ns; i++) CK(hipStreamWaitEvent(ds[i], kd, 0));
            for (int i = 0; i < m; i++)
                CK(hipMemcpyAsync(sep[i].data(), d + (k + i) * B, B, hipMemcpyDeviceToHost, ds[i % ns]));
            for (int i = 0; i < ns; i++) CK(hipStreamSynchronize(ds[i]));
        });
    }
    bench("(i) per-block D2H alone, 1 stream (separate)", [&] {
        for (int i = 0; i < m; i++) CK(hipMemcpyAsync(sep[i].data(), d + (k + i) * B, B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    bench("(i') one D2H of 4 MiB alone (contiguous)", [&] {
        CK(hipMemcpyAsync(coding.data(), d + k * B, m * B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    bench("(i'') per-block D2H alone, hipMemcpy (sync) each", [&] {
        for (int i = 0; i < m; i++) CK(hipMemcpy(sep[i].data(), d + (k + i) * B, B, hipMemcpyDeviceToHost));
    });
    bench("(b) hipHostRegister + DMA + unregister", [&] {
        CK(hipHostRegister(value.data(), k * B, hipHostRegisterDefault));
        CK(hipHostRegister(coding.data(), m * B, hipHostRegisterDefault));
        CK(hipMemcpyAsync(d, value.data(), k * B, hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(coding.data(), d + k * B, m * B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        CK(hipHostUnregister(value.data()));
        CK(hipHostUnregister(coding.data()));
    });
    for (int T : {1, 4, 8, 16}) {
        char nm[80];
        snprintf(nm, sizeof nm, "(c) %2d-thread memcpy to pinned + one DMA each way", T);
        bench(nm, [&] {
            par_memcpy(pin, value.data(), k * B, T);
            CK(hipMemcpyAsync(d, pin, k * B, hipMemcpyHostToDevice, st));
            CK(hipMemcpyAsync(pin + k * B, d + k * B, m * B, hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            par_memcpy(coding.data(), pin + k * B, m * B, T);
        });
    }
    {
        // (j) per-block D2H copies issued from m persistent host threads, one stream each (a pageable copy
        // blocks its issuing thread, so one thread runs the staged copies one after the other)
        std::atomic<int> gen{0}, done{0};
        std::atomic<bool> quit{false};
        hipEvent_t ready;
        CK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        std::vector<std::thread> pool;
        for (int i = 0; i < m; i++)
            pool.emplace_back([&, i] {
                CK(hipSetDevice(0));
                int seen = 0;
                while (true) {
                    int g;
                    while ((g = gen.load(std::memory_order_acquire)) == seen && !quit.load()) {}
                    if (quit.load()) return;
                    seen = g;
                    CK(hipStreamWaitEvent(ds[i], ready, 0));
                    CK(hipMemcpyAsync(sep[i].data(), d + (k + i) * B, B, hipMemcpyDeviceToHost, ds[i]));
                    CK(hipStreamSynchronize(ds[i]));
                    done.fetch_add(1, std::memory_order_acq_rel);
                }
            });
        bench("(j) one H2D + per-block D2H from m host threads", [&] {
            CK(hipMemcpyAsync(d, value.data(), k * B, hipMemcpyHostToDevice, st));
            CK(hipEventRecord(ready, st));
            done.store(0);
            gen.fetch_add(1, std::memory_order_acq_rel);
            while (done.load(std::memory_order_acquire) < m) {}
        });
        bench("(j') per-block D2H alone from m host threads", [&] {
            CK(hipEventRecord(ready, st));
            done.store(0);
            gen.fetch_add(1, std::memory_order_acq_rel);
            while (done.load(std::memory_order_acquire) < m) {}
        });
        quit.store(true);
        for (auto& t : pool) t.join();
    }
    bench("pinned DMA only (lower bound)", [&] {
        CK(hipMemcpyAsync(d, pin, k * B, hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(pin + k * B, d + k * B, m * B, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    return 0;
}
