// Build: hipcc -O1 -g -std=c++17 --offload-arch=gfx950 profiles/r04/stream/stream_lifetime_probe.cpp -o profiles/r04/stream/stream_lifetime_probe
// What the HIP runtime does with a stream handle or an event after hipStreamDestroy:
// one case per process (a case may crash; the runner starts each under its own timeout).
//   1 query_after_destroy   event recorded on S (work queued), S destroyed, then query / sync the event
//   2 record_on_destroyed   S destroyed (handle not reused), then hipEventRecord(E, S)
//   3 wait_on_stale_event   event recorded on S1, S1 destroyed, S2 created, hipStreamWaitEvent(S2, E)
//   4 record_on_reused      S1 destroyed, S2 created (same handle?), hipEventRecord(E, S1 handle)
//   5 query_destroyed       S destroyed, hipStreamQuery(S)
//   6 rerecord_after_destroy event recorded on S1, S1 destroyed, the SAME event re-recorded on S2, queried
//   7 wait_on_destroyed     S destroyed, hipStreamWaitEvent(S, E)
//   8 record_cost           host cost of hipEventRecord / hipMemsetAsync / hipEventQuery per call
//   9 record_gpu_cost       GPU time of 4096 back-to-back small kernels with an event recorded behind each,
//                           by event flags (none / default / no system fence / release to device / every 64th)
//  10 ext_stop_event        the same with the event bound to the launch (hipExtLaunchKernel stopEvent), by flags;
//                           then: stop event of a launch on S1, S1 destroyed, event queried
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define STEP(what, call)                                                                          \
    do {                                                                                          \
        printf("  %-44s ", what);                                                                 \
        fflush(stdout);                                                                           \
        hipError_t _e = (call);                                                                   \
        printf("-> %d (%s)\n", (int)_e, hipGetErrorName(_e));                                     \
        fflush(stdout);                                                                           \
    } while (0)

__global__ void touch_kernel(uint4* p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = make_uint4(i, i + 1, i + 2, i + 3);
}

int main(int argc, char** argv) {
    const int c = argc > 1 ? atoi(argv[1]) : 1;
    void* buf = nullptr;
    const size_t bytes = 256u << 20;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 2;
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    hipStream_t s1 = nullptr, s2 = nullptr;
    printf("case %d\n", c);
    switch (c) {
    case 1:
        STEP("create S1", hipStreamCreate(&s1));
        for (int i = 0; i < 8; i++) (void)hipMemsetAsync(buf, i, bytes, s1);
        STEP("record E on S1", hipEventRecord(e, s1));
        STEP("destroy S1", hipStreamDestroy(s1));
        STEP("query E", hipEventQuery(e));
        STEP("synchronize E", hipEventSynchronize(e));
        break;
    case 2:
        STEP("create S1", hipStreamCreate(&s1));
        STEP("destroy S1", hipStreamDestroy(s1));
        STEP("record E on destroyed S1", hipEventRecord(e, s1));
        STEP("get last error", hipGetLastError());
        STEP("query E", hipEventQuery(e));
        break;
    case 3:
        STEP("create S1", hipStreamCreate(&s1));
        for (int i = 0; i < 8; i++) (void)hipMemsetAsync(buf, i, bytes, s1);
        STEP("record E on S1", hipEventRecord(e, s1));
        STEP("destroy S1", hipStreamDestroy(s1));
        STEP("create S2", hipStreamCreate(&s2));
        printf("  handles S1 %p S2 %p\n", (void*)s1, (void*)s2);
        STEP("S2 waits for E", hipStreamWaitEvent(s2, e, 0));
        STEP("memset on S2", hipMemsetAsync(buf, 1, bytes, s2));
        STEP("synchronize S2", hipStreamSynchronize(s2));
        STEP("destroy S2", hipStreamDestroy(s2));
        break;
    case 4:
        STEP("create S1", hipStreamCreate(&s1));
        STEP("destroy S1", hipStreamDestroy(s1));
        STEP("create S2", hipStreamCreate(&s2));
        printf("  handles S1 %p S2 %p\n", (void*)s1, (void*)s2);
        STEP("record E on S1 handle", hipEventRecord(e, s1));
        STEP("synchronize E", hipEventSynchronize(e));
        STEP("destroy S2", hipStreamDestroy(s2));
        break;
    case 5:
        STEP("create S1", hipStreamCreate(&s1));
        STEP("destroy S1", hipStreamDestroy(s1));
        STEP("query destroyed S1", hipStreamQuery(s1));
        STEP("get last error", hipGetLastError());
        break;
    case 6:
        STEP("create S1", hipStreamCreate(&s1));
        for (int i = 0; i < 8; i++) (void)hipMemsetAsync(buf, i, bytes, s1);
        STEP("record E on S1", hipEventRecord(e, s1));
        STEP("destroy S1", hipStreamDestroy(s1));
        STEP("create S2", hipStreamCreate(&s2));
        (void)hipMemsetAsync(buf, 3, bytes, s2);
        STEP("re-record E on S2", hipEventRecord(e, s2));
        STEP("query E", hipEventQuery(e));
        STEP("synchronize E", hipEventSynchronize(e));
        STEP("destroy S2", hipStreamDestroy(s2));
        break;
    case 7:
        STEP("create S1", hipStreamCreate(&s1));
        STEP("destroy S1", hipStreamDestroy(s1));
        STEP("record E on null stream", hipEventRecord(e, nullptr));
        STEP("destroyed S1 waits for E", hipStreamWaitEvent(s1, e, 0));
        STEP("get last error", hipGetLastError());
        break;
    case 8: {  // host cost of hipEventRecord per call (the price of a completion event per launch)
        STEP("create S1", hipStreamCreate(&s1));
        hipEvent_t ev[16];
        for (auto& x : ev) (void)hipEventCreateWithFlags(&x, hipEventDisableTiming);
        for (int rep = 0; rep < 3; rep++) {
            const int N = 20000;
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; i++) (void)hipEventRecord(ev[i & 15], s1);
            auto t1 = std::chrono::steady_clock::now();
            (void)hipStreamSynchronize(s1);
            auto t2 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; i++) (void)hipMemsetAsync(buf, 0, 64, s1);
            auto t3 = std::chrono::steady_clock::now();
            (void)hipStreamSynchronize(s1);
            auto t4 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; i++) {
                (void)hipMemsetAsync(buf, 0, 64, s1);
                (void)hipEventRecord(ev[i & 15], s1);
            }
            auto t5 = std::chrono::steady_clock::now();
            (void)hipStreamSynchronize(s1);
            auto t6 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; i++) (void)hipEventQuery(ev[i & 15]);
            auto t7 = std::chrono::steady_clock::now();
            auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            printf("  rep %d: record %.3f us, memset %.3f us, memset+record %.3f us, query %.3f us (per call)\n",
                   rep, us(t0, t1) / N, us(t2, t3) / N, us(t4, t5) / N, us(t6, t7) / N);
            fflush(stdout);
        }
        STEP("destroy S1", hipStreamDestroy(s1));
        for (auto& x : ev) (void)hipEventDestroy(x);
        break;
    }
    case 9: {
        STEP("create S1", hipStreamCreate(&s1));
        const unsigned fl[5] = {0, hipEventDisableTiming, hipEventDisableTiming | hipEventDisableSystemFence,
                                hipEventDisableTiming | hipEventReleaseToDevice, hipEventDisableTiming};
        const char* names[5] = {"none", "default", "no-system-fence", "release-to-device", "every-64th"};
        hipEvent_t t0, t1;
        (void)hipEventCreate(&t0);
        (void)hipEventCreate(&t1);
        const int N = 4096, n = 4096;  // 64 KiB written per kernel
        for (int rep = 0; rep < 2; rep++)
            for (int v = 0; v < 5; v++) {
                hipEvent_t ev[8];
                for (auto& x : ev) (void)hipEventCreateWithFlags(&x, v ? fl[v] : hipEventDisableTiming);
                (void)hipStreamSynchronize(s1);
                auto h0 = std::chrono::steady_clock::now();
                (void)hipEventRecord(t0, s1);
                for (int i = 0; i < N; i++) {
                    hipLaunchKernelGGL(touch_kernel, dim3(n / 256), dim3(256), 0, s1, (uint4*)buf, n);
                    if (v == 1 || v == 2 || v == 3 || (v == 4 && (i & 63) == 63)) (void)hipEventRecord(ev[i & 7], s1);
                }
                (void)hipEventRecord(t1, s1);
                auto h1 = std::chrono::steady_clock::now();
                (void)hipEventSynchronize(t1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, t0, t1);
                printf("  rep %d %-18s GPU %.3f us/launch, host %.3f us/launch\n", rep, names[v], ms * 1e3 / N,
                       std::chrono::duration<double, std::micro>(h1 - h0).count() / N);
                fflush(stdout);
                for (auto& x : ev) (void)hipEventDestroy(x);
            }
        STEP("destroy S1", hipStreamDestroy(s1));
        break;
    }
    case 10: {
        STEP("create S1", hipStreamCreate(&s1));
        const unsigned fl[4] = {hipEventDisableTiming, hipEventDisableTiming, hipEventDisableTiming | hipEventDisableSystemFence,
                                hipEventDisableTiming | hipEventReleaseToDevice};
        const char* names[4] = {"plain launch", "ext stop default", "ext stop no-sys-fence", "ext stop rel-to-device"};
        hipEvent_t t0, t1;
        (void)hipEventCreate(&t0);
        (void)hipEventCreate(&t1);
        const int N = 4096;
        int n = 4096;
        uint4* p = (uint4*)buf;
        void* args[] = {&p, &n};
        for (int rep = 0; rep < 2; rep++)
            for (int v = 0; v < 4; v++) {
                hipEvent_t ev[8];
                for (auto& x : ev) (void)hipEventCreateWithFlags(&x, fl[v]);
                (void)hipStreamSynchronize(s1);
                auto h0 = std::chrono::steady_clock::now();
                (void)hipEventRecord(t0, s1);
                for (int i = 0; i < N; i++) {
                    if (v == 0)
                        (void)hipLaunchKernel((const void*)touch_kernel, dim3(n / 256), dim3(256), args, 0, s1);
                    else
                        (void)hipExtLaunchKernel((const void*)touch_kernel, dim3(n / 256), dim3(256), args, 0, s1,
                                                 nullptr, ev[i & 7], 0);
                }
                (void)hipEventRecord(t1, s1);
                auto h1 = std::chrono::steady_clock::now();
                (void)hipEventSynchronize(t1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, t0, t1);
                printf("  rep %d %-24s GPU %.3f us/launch, host %.3f us/launch, last event query %d\n", rep, names[v],
                       ms * 1e3 / N, std::chrono::duration<double, std::micro>(h1 - h0).count() / N,
                       (int)hipEventQuery(ev[(N - 1) & 7]));
                fflush(stdout);
                for (auto& x : ev) (void)hipEventDestroy(x);
            }
        for (int v = 1; v < 4; v++) {
            hipEvent_t ev;
            (void)hipEventCreateWithFlags(&ev, fl[v]);
            hipStream_t s3 = nullptr;
            STEP("create S3", hipStreamCreate(&s3));
            for (int i = 0; i < 64; i++) (void)hipMemsetAsync(buf, i, bytes, s3);
            STEP("ext launch with stop event on S3", hipExtLaunchKernel((const void*)touch_kernel, dim3(n / 256), dim3(256), args, 0, s3, nullptr, ev, 0));
            STEP("query stop event (work queued)", hipEventQuery(ev));
            STEP("destroy S3", hipStreamDestroy(s3));
            STEP("query stop event after destroy", hipEventQuery(ev));
            STEP("synchronize stop event", hipEventSynchronize(ev));
            (void)hipEventDestroy(ev);
        }
        STEP("destroy S1", hipStreamDestroy(s1));
        break;
    }
    default:
        return 2;
    }
    STEP("device synchronize", hipDeviceSynchronize());
    (void)hipEventDestroy(e);
    (void)hipFree(buf);
    printf("case %d done\n", c);
    return 0;
}
