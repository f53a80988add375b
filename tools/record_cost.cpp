// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -Iinclude tools/record_cost.cpp -Lerasure-codes-prototype_amd/lib -lecg
//        -Wl,-rpath,'$ORIGIN/../erasure-codes-prototype_amd/lib' -o tools/record_cost
// Batch-scope record cost on the GPU box: per-call host time of recording ecg_ec_encode inside a scope
// (real HBM blocks), and the cost of the HIP calls on that path.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include "ecg.h"
static double us(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}
int main() {
    const int k = 10, m = 4, n = 14, S = 4096;
    const long long B = 65536;
    uint8_t* buf = nullptr;
    if (hipMalloc(&buf, (size_t)S * n * B) != hipSuccess) return 1;
    std::vector<char*> ptrs((size_t)S * n);
    for (size_t i = 0; i < ptrs.size(); i++) ptrs[i] = (char*)(buf + i * B);
    ecg_coding_parameters cp{};
    cp.k = k; cp.m = m;
    ecg_ec* ec = ecg_ec_factory(ECG_RS, &cp);
    ecg_ec_set_memory(ec, ECG_MEM_DEVICE, nullptr);
    for (int rep = 0; rep < 4; rep++) {
        ecg_batch_begin();
        auto t0 = std::chrono::steady_clock::now();
        for (int s = 0; s < S; s++) ecg_ec_encode(ec, &ptrs[(size_t)s * n], &ptrs[(size_t)s * n + k], (int)B);
        auto t1 = std::chrono::steady_clock::now();
        int rc = ecg_batch_end();
        (void)hipDeviceSynchronize();
        printf("record %.3f us/call (flush rc %d)\n", us(t0, t1) / S, rc);
    }
    int d = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 100000; i++) (void)hipGetDevice(&d);
    auto t1 = std::chrono::steady_clock::now();
    printf("hipGetDevice %.3f us/call\n", us(t0, t1) / 100000);
    (void)hipFree(buf);
    return 0;
}
