// Where the time of a deferred host-tier batch goes (tuning probe, not shipped): config 1's SET loop --
// one jerasure_matrix_encode per RS(6,4) stripe on host buffers -- inside a batch scope with host deferral
// (ecg_batch_defer_host).  Reports the host time per recorded call and the time of the flush at
// ecg_batch_end (one H2D, the grouped launches, one D2H, the scatter into the caller's buffers).
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -Iinclude profiles/r04/small_host/defer_cost.cpp -Lerasure-codes-prototype_amd/lib -lecg
//        -Wl,-rpath,'$ORIGIN/../erasure-codes-prototype_amd/lib' -o profiles/r04/small_host/defer_cost
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ecg.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const int k = 6, m = 4;
    int* M = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
    for (int B : {1024, 4096}) {
        for (int S : {64, 4096}) {
            std::vector<char> data((size_t)S * k * B), coding((size_t)S * m * B);
            for (size_t i = 0; i < data.size(); i++) data[i] = (char)(i * 131 + 7);
            std::vector<char*> dp(k), cp(m);
            double best_rec = 1e30, best_end = 1e30;
            for (int rep = 0; rep < 6; rep++) {
                if (ecg_batch_begin() || ecg_batch_defer_host(1)) return 1;
                const double t0 = now_us();
                for (int s = 0; s < S; s++) {
                    for (int j = 0; j < k; j++) dp[j] = data.data() + ((size_t)s * k + j) * B;
                    for (int j = 0; j < m; j++) cp[j] = coding.data() + ((size_t)s * m + j) * B;
                    if (ecg_jerasure_matrix_encode(k, m, 8, M, dp.data(), cp.data(), B)) return 2;
                }
                const double t1 = now_us();
                if (ecg_batch_end()) return 3;
                const double t2 = now_us();
                if (rep > 0) {
                    best_rec = std::min(best_rec, (t1 - t0) / S);
                    best_end = std::min(best_end, t2 - t1);
                }
            }
            printf("RS(6,4) B=%5d S=%5d: record %.3f us/call, flush %.1f us (%.3f us/stripe), total %.3f us/stripe\n",
                   B, S, best_rec, best_end, best_end / S, best_rec + best_end / S);
            fflush(stdout);
        }
    }
    ecg_free(M);
    return 0;
}
