// ThreadSanitizer driver of the engine's concurrency (TEST INFRASTRUCTURE; tools/tsan_host.sh builds it
// against tests/tsan/hip_stub.cpp, tests/test_sanitize.py runs it).
//
// The reference runs each EC call on a detached thread (proxy.cpp:416-419).  Here T threads each issue a
// random sequence of the calls a proxy makes, through the C ABI (include/ecg.h), at once:
//   * device-tier encodes and decodes on the thread's own stream, hipStreamPerThread or the null stream,
//     with coefficient matrices drawn from a pool larger than the program cache (ECG_OPT_PROGRAM_CACHE = 4),
//     so program sets are evicted, retired, covered and reclaimed while other threads launch from them;
//   * batch scopes with scratch partials (a helper partial + main partial + perform_addition repair), and
//     with deferred host-tier calls (ecg_batch_defer_host);
//   * synchronous host-tier calls (zero-copy staging with completion flags, pooled host contexts);
//   * host-resident batch pipelines; the ErasureCode facade on host blocks; repair planning;
//   * stream churn (the thread's stream destroyed and a new one created), explicit reclaims, option changes;
//   * two devices: a quarter of the operations run on device 1, and scopes record calls on both devices.
// Every result is compared with the oracle (oracle/jerasure_w8.c); the kernels run on the CPU in the stub,
// bit-exact.  Exit status: 0 when every check passed; ThreadSanitizer reports go to stderr (the test treats
// any report as a failure).
// Usage: engine_race [threads=8] [ops=150] [seed=1]
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <unistd.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "ecg.h"

extern "C" {
void orc_matrix_encode(int k, int m, const int* matrix, uint8_t** data, uint8_t** coding, long size);
int* orc_reed_sol_vandermonde_coding_matrix(int k, int m);
void orc_free(void* p);
void hip_stub_stall(hipStream_t st, int ms);  // tests/tsan/hip_stub.cpp test hooks
long hip_stub_hazards();
long hip_stub_not_ready();
}

namespace {

std::atomic<int> g_fail{0};
std::atomic<long> g_checks{0};
std::atomic<const char*> g_doing[64];  // what each thread is doing (the watchdog prints it)
std::atomic<int> g_max_retiring{0};    // the most evicted program sets seen waiting for retirement at once

#define CHECK(cond, ...)                                  \
    do {                                                  \
        g_checks++;                                       \
        if (!(cond)) {                                    \
            fprintf(stderr, "CHECK FAILED %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fprintf(stderr, "\n");                        \
            g_fail++;                                     \
        }                                                 \
    } while (0)

constexpr int K = 4, M = 2;
std::vector<std::vector<int>> g_mats;  // the matrix pool (read-only once the threads start)

void* dmalloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, n) != hipSuccess) abort();
    return p;
}

void expect_encode(const std::vector<int>& mat, int k, int m, std::vector<uint8_t*> data, std::vector<uint8_t*> got,
                   long B, const char* what) {
    std::vector<std::vector<uint8_t>> want(m, std::vector<uint8_t>(B));
    std::vector<uint8_t*> wp(m);
    for (int i = 0; i < m; i++) wp[i] = want[i].data();
    orc_matrix_encode(k, m, mat.data(), data.data(), wp.data(), B);
    for (int i = 0; i < m; i++) CHECK(memcmp(want[i].data(), got[i], B) == 0, "%s: output %d differs", what, i);
}

constexpr int kDev = 2;  // the HIP stand-in's devices

struct Worker {
    int tid;
    std::mt19937_64 rng;
    hipStream_t owns[kDev] = {};
    hipStream_t own = nullptr;  // the thread's stream on its current device
    int dev = 0;
    explicit Worker(int t, unsigned long long seed) : tid(t), rng(seed * 1000003ull + t) {}

    int pick(int n) { return (int)(rng() % (unsigned long long)n); }
    void use_device(int d) {  // the thread's device for the next operation (its buffers and streams follow)
        dev = d;
        CHECK(ecg_set_device(d) == 0, "set_device %d", d);
        own = owns[d];
    }
    void fill(uint8_t* p, long n) {
        for (long i = 0; i < n; i++) p[i] = (uint8_t)rng();
    }
    hipStream_t stream() {
        switch (pick(4)) {
            case 0: return hipStreamPerThread;
            case 1: return nullptr;
            default: return own;
        }
    }
    long block() {
        static const long sizes[] = {64, 1000, 4096, 4096 + 16, 16384};
        return sizes[pick(5)];
    }

    // device-tier encode (ecg_dev_matrix_encode) on a random stream
    void dev_encode() {
        const std::vector<int>& mat = g_mats[pick((int)g_mats.size())];
        const long B = block();
        std::vector<uint8_t> host((size_t)K * B);
        fill(host.data(), (long)host.size());
        uint8_t* d = (uint8_t*)dmalloc((size_t)(K + M) * B);
        hipStream_t st = stream();
        hipMemcpyAsync(d, host.data(), (size_t)K * B, hipMemcpyHostToDevice, st);
        std::vector<char*> dp(K), cp(M);
        for (int j = 0; j < K; j++) dp[j] = (char*)d + (size_t)j * B;
        for (int i = 0; i < M; i++) cp[i] = (char*)d + (size_t)(K + i) * B;
        CHECK(ecg_dev_matrix_encode(K, M, mat.data(), dp.data(), cp.data(), B, st) == 0, "dev encode rc");
        hipStreamSynchronize(st);
        std::vector<uint8_t*> in(K), out(M);
        for (int j = 0; j < K; j++) in[j] = host.data() + (size_t)j * B;
        for (int i = 0; i < M; i++) out[i] = (uint8_t*)cp[i];
        expect_encode(mat, K, M, in, out, B, "dev encode");
        hipFree(d);
    }

    // device-tier decode of RS(6,3) with one or two erasures (ecg_dev_matrix_decode, row_k_ones = failed_num)
    void dev_decode() {
        const int k = 6, m = 3;
        int* mat = orc_reed_sol_vandermonde_coding_matrix(k, m);
        const long B = block();
        std::vector<uint8_t> host((size_t)(k + m) * B);
        fill(host.data(), (long)k * B);
        std::vector<uint8_t*> in(k), par(m);
        for (int j = 0; j < k; j++) in[j] = host.data() + (size_t)j * B;
        for (int i = 0; i < m; i++) par[i] = host.data() + (size_t)(k + i) * B;
        orc_matrix_encode(k, m, mat, in.data(), par.data(), B);
        uint8_t* d = (uint8_t*)dmalloc(host.size());
        hipStream_t st = stream();
        hipMemcpyAsync(d, host.data(), host.size(), hipMemcpyHostToDevice, st);
        const int nf = 1 + pick(2);
        int er[3] = {pick(k + m), -1, -1};
        if (nf == 2) er[1] = (er[0] + 1 + pick(k + m - 1)) % (k + m);
        std::vector<char*> dp(k), cp(m);
        for (int j = 0; j < k; j++) dp[j] = (char*)d + (size_t)j * B;
        for (int i = 0; i < m; i++) cp[i] = (char*)d + (size_t)(k + i) * B;
        for (int f = 0; f < nf; f++) hipMemsetAsync(d + (size_t)er[f] * B, 0xA5, B, st);  // poisoned
        CHECK(ecg_dev_matrix_decode(k, m, mat, nf, er, dp.data(), cp.data(), B, st) == 0, "dev decode rc");
        hipStreamSynchronize(st);
        CHECK(memcmp(d, host.data(), host.size()) == 0, "dev decode: stripe differs after decoding {%d,%d}", er[0],
              er[1]);
        hipFree(d);
        orc_free(mat);
    }

    // a repair as the proxies issue it, in a batch scope with the partials declared scratch:
    // p0 = row(d0, d1), p1 = row(d2, d3), out = p0 ^ p1 (perform_addition)
    void scope_repair() {
        const std::vector<int>& mat = g_mats[pick((int)g_mats.size())];
        const long B = block();
        const int S = 1 + pick(6);
        hipStream_t st = own;
        std::vector<uint8_t> host((size_t)S * K * B);
        fill(host.data(), (long)host.size());
        uint8_t* d = (uint8_t*)dmalloc(host.size());
        uint8_t* parts = (uint8_t*)dmalloc((size_t)S * 2 * B);
        uint8_t* out = (uint8_t*)dmalloc((size_t)S * B);
        hipMemcpyAsync(d, host.data(), host.size(), hipMemcpyHostToDevice, st);
        CHECK(ecg_batch_begin() == 0, "batch_begin");
        if (pick(2)) CHECK(ecg_batch_scratch(parts, (size_t)S * 2 * B) == 0, "batch_scratch");
        const int ones[2] = {1, 1};
        for (int s = 0; s < S; s++) {
            char* blk[K];
            for (int j = 0; j < K; j++) blk[j] = (char*)d + ((size_t)s * K + j) * B;
            char* p[2] = {(char*)parts + (size_t)(2 * s) * B, (char*)parts + (size_t)(2 * s + 1) * B};
            char* o = (char*)out + (size_t)s * B;
            CHECK(ecg_dev_matrix_encode(2, 1, &mat[0], blk, &p[0], B, st) == 0, "helper partial");
            CHECK(ecg_dev_matrix_encode(2, 1, &mat[2], blk + 2, &p[1], B, st) == 0, "main partial");
            CHECK(ecg_dev_matrix_encode(2, 1, ones, p, &o, B, st) == 0, "perform_addition");
        }
        CHECK(ecg_batch_end() == 0, "batch_end");
        hipStreamSynchronize(st);
        const std::vector<int> row = {mat[0], mat[1], mat[2], mat[3]};
        for (int s = 0; s < S; s++) {
            std::vector<uint8_t*> in(K);
            for (int j = 0; j < K; j++) in[j] = host.data() + ((size_t)s * K + j) * B;
            std::vector<uint8_t*> got = {out + (size_t)s * B};
            expect_encode(row, K, 1, in, got, B, "scope repair");
        }
        hipFree(d);
        hipFree(parts);
        hipFree(out);
    }

    // host-tier calls (ecg_jerasure_matrix_encode on host buffers), optionally deferred in a scope
    void host_encode(bool deferred) {
        const std::vector<int>& mat = g_mats[pick((int)g_mats.size())];
        const long B = block();
        const int n = deferred ? 1 + pick(8) : 1;
        std::vector<std::vector<uint8_t>> data(n, std::vector<uint8_t>((size_t)K * B)),
            coding(n, std::vector<uint8_t>((size_t)M * B));
        if (deferred) {
            CHECK(ecg_batch_begin() == 0, "batch_begin");
            CHECK(ecg_batch_defer_host(1) == 0, "defer_host");
        }
        for (int c = 0; c < n; c++) {
            fill(data[c].data(), (long)data[c].size());
            char* dp[K];
            char* cp[M];
            for (int j = 0; j < K; j++) dp[j] = (char*)data[c].data() + (size_t)j * B;
            for (int i = 0; i < M; i++) cp[i] = (char*)coding[c].data() + (size_t)i * B;
            CHECK(ecg_jerasure_matrix_encode(K, M, 8, const_cast<int*>(mat.data()), dp, cp, (int)B) == 0, "host encode");
        }
        if (deferred) CHECK(ecg_batch_end() == 0, "batch_end");
        for (int c = 0; c < n; c++) {
            std::vector<uint8_t*> in(K), out(M);
            for (int j = 0; j < K; j++) in[j] = data[c].data() + (size_t)j * B;
            for (int i = 0; i < M; i++) out[i] = coding[c].data() + (size_t)i * B;
            expect_encode(mat, K, M, in, out, B, deferred ? "deferred host encode" : "host encode");
        }
    }

    // host-resident batch through the 3-stream pipeline (ecg_encode_batch_host)
    void host_pipeline() {
        const std::vector<int>& mat = g_mats[pick((int)g_mats.size())];
        const long B = 4096;
        const int S = 3 + pick(6);
        std::vector<uint8_t> st((size_t)S * (K + M) * B);
        fill(st.data(), (long)st.size());
        CHECK(ecg_encode_batch_host(K, M, mat.data(), st.data(), (K + M) * B, B, st.data() + (size_t)K * B, (K + M) * B,
                                    B, B, S, 2) == 0,
              "encode_batch_host");
        for (int s = 0; s < S; s++) {
            std::vector<uint8_t*> in(K), out(M);
            for (int j = 0; j < K; j++) in[j] = st.data() + ((size_t)s * (K + M) + j) * B;
            for (int i = 0; i < M; i++) out[i] = st.data() + ((size_t)s * (K + M) + K + i) * B;
            expect_encode(mat, K, M, in, out, B, "host pipeline");
        }
    }

    // ErasureCode facade on host blocks: Azure-LRC(12,2,2) encode, then a repair plan (planning code)
    void facade() {
        ecg_coding_parameters cp;
        memset(&cp, 0, sizeof(cp));
        cp.k = 12;
        cp.l = 2;
        cp.g = 2;
        cp.local_or_column = 1;
        ecg_ec* ec = ecg_ec_factory(ECG_AZURE_LRC, &cp);
        CHECK(ec != nullptr, "ec_factory");
        if (!ec) return;
        ecg_ec_init_coding_parameters(ec, &cp);
        const long B = 1024;
        std::vector<uint8_t> blocks((size_t)16 * B);
        fill(blocks.data(), 12 * B);
        char* dp[12];
        char* cpp[4];
        for (int j = 0; j < 12; j++) dp[j] = (char*)blocks.data() + (size_t)j * B;
        for (int i = 0; i < 4; i++) cpp[i] = (char*)blocks.data() + (size_t)(12 + i) * B;
        CHECK(ecg_ec_encode(ec, dp, cpp, (int)B) == 0, "facade encode");
        std::vector<int> fm(4 * 12);
        CHECK(ecg_ec_make_encoding_matrix(ec, fm.data()) == 0, "facade matrix");
        std::vector<uint8_t*> in(12), out(4);
        for (int j = 0; j < 12; j++) in[j] = (uint8_t*)dp[j];
        for (int i = 0; i < 4; i++) out[i] = (uint8_t*)cpp[i];
        expect_encode(fm, 12, 4, in, out, B, "facade encode");
        ecg_ec_generate_partition(ec);
        const int fail = pick(16);
        int buf[512], decodable = 0;
        CHECK(ecg_ec_generate_repair_plan(ec, &fail, 1, buf, 512, &decodable) >= 0, "repair plan");
        ecg_ec_destroy(ec);
    }

    void churn() {
        if (owns[dev]) {
            hipStreamSynchronize(owns[dev]);
            hipStreamDestroy(owns[dev]);
        }
        hipStreamCreate(&owns[dev]);
        own = owns[dev];
    }

    // one scope whose calls alternate between the two devices, each on that device's stream: every group
    // must launch on the device its calls were recorded on, whatever the thread's device at the flush
    void two_device_scope() {
        const long B = 4096;
        const int S = 2 + pick(5);
        std::vector<std::vector<uint8_t>> host(S, std::vector<uint8_t>((size_t)K * B));
        std::vector<uint8_t*> d(S);
        std::vector<int> devs(S), mats(S);
        for (int s = 0; s < S; s++) {
            devs[s] = s % kDev;
            mats[s] = pick((int)g_mats.size());
            use_device(devs[s]);
            fill(host[s].data(), (long)host[s].size());
            d[s] = (uint8_t*)dmalloc((size_t)(K + M) * B);
            hipMemcpyAsync(d[s], host[s].data(), (size_t)K * B, hipMemcpyHostToDevice, own);
            hipStreamSynchronize(own);
        }
        CHECK(ecg_batch_begin() == 0, "batch_begin");
        for (int s = 0; s < S; s++) {
            use_device(devs[s]);
            char* dp[K];
            char* cp[M];
            for (int j = 0; j < K; j++) dp[j] = (char*)d[s] + (size_t)j * B;
            for (int i = 0; i < M; i++) cp[i] = (char*)d[s] + (size_t)(K + i) * B;
            CHECK(ecg_dev_matrix_encode(K, M, g_mats[mats[s]].data(), dp, cp, B, own) == 0, "2-device record");
        }
        use_device(pick(kDev));
        CHECK(ecg_batch_end() == 0, "batch_end (2 devices)");
        for (int s = 0; s < S; s++) {
            use_device(devs[s]);
            hipStreamSynchronize(own);
            std::vector<uint8_t*> in(K), out(M);
            for (int j = 0; j < K; j++) in[j] = host[s].data() + (size_t)j * B;
            for (int i = 0; i < M; i++) out[i] = d[s] + (size_t)(K + i) * B;
            expect_encode(g_mats[mats[s]], K, M, in, out, B, "two-device scope");
            hipFree(d[s]);
        }
    }

    void run(int ops) {
        for (int d = 0; d < kDev; d++) {
            use_device(d);
            hipStreamCreate(&owns[d]);
        }
        auto& doing = g_doing[tid & 63];
        for (int i = 0; i < ops; i++) {
            use_device(pick(4) == 0 ? 1 : 0);  // device 1 for a quarter of the operations
            switch (pick(17)) {
                case 0: case 1: case 2: case 3: doing = "dev_encode"; dev_encode(); break;
                case 4: case 5: doing = "dev_decode"; dev_decode(); break;
                case 6: case 7: case 8: doing = "scope_repair"; scope_repair(); break;
                case 9: doing = "host_encode"; host_encode(false); break;
                case 10: case 11: doing = "deferred host_encode"; host_encode(true); break;
                case 12: doing = "host_pipeline"; host_pipeline(); break;
                case 13: doing = "facade"; facade(); break;
                case 14: doing = "churn"; churn(); break;
                case 15: doing = "two_device_scope"; two_device_scope(); break;
                default:
                    doing = "reclaim / options";
                    if (pick(2)) ecg_program_sets_reclaim();
                    else ecg_set_option(ECG_OPT_PROGRAM_CACHE, 4 + 2 * pick(2));
                    {
                        const int r = ecg_program_sets_retiring();
                        int seen = g_max_retiring.load();
                        while (r > seen && !g_max_retiring.compare_exchange_weak(seen, r)) {
                        }
                    }
                    (void)ecg_program_cache_size();
                    break;
            }
        }
        doing = "done";
        for (int d = 0; d < kDev; d++) {
            use_device(d);
            hipStreamSynchronize(owns[d]);
            hipStreamDestroy(owns[d]);
        }
    }
};

// hipStreamPerThread names a different stream on every thread.  Thread A builds program set P_A
// (a call, synchronized), queues 300 ms of device time on ITS per-thread stream, then calls P_A again: the
// launch, noted under that handle, waits behind the queue.  Thread B, on
// ITS per-thread stream, evicts P_A (cache of 2) with twelve new programs, synchronizing after each.  If B
// could cover P_A on B's stream, the cover would fire at once, P_A's tables would go back to the pool and
// B's next upload would overwrite them while A's launch still reads them: the stub reports that as a
// device-time hazard (its data effects happen at enqueue, so only the hazard check can see it).
void per_thread_scenario() {
    const long B = 4096;
    const long before = hip_stub_hazards();
    ecg_set_option(ECG_OPT_PROGRAM_CACHE, 2);
    std::vector<uint8_t> host((size_t)K * B);
    std::mt19937_64 rng(99);
    for (auto& x : host) x = (uint8_t)rng();
    uint8_t* d = (uint8_t*)dmalloc((size_t)(K + 2 * M * 13) * B);
    if (hipMemcpy(d, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) abort();
    std::vector<std::vector<int>> mats;
    for (int i = 0; i < 13; i++) {
        std::vector<int> m(K * M);
        for (int& c : m) c = 2 + (int)(rng() % 254);
        mats.push_back(m);
    }
    auto call = [&](int i) {
        char* dp[K];
        char* cp[M];
        for (int j = 0; j < K; j++) dp[j] = (char*)d + (size_t)j * B;
        for (int p = 0; p < M; p++) cp[p] = (char*)d + (size_t)(K + M * i + p) * B;
        CHECK(ecg_dev_matrix_encode(K, M, mats[i].data(), dp, cp, B, hipStreamPerThread) == 0, "per-thread call %d", i);
    };
    std::atomic<int> stage{0};
    std::thread a([&] {
        call(0);  // P_A built and its upload complete: only the launch below holds its tables
        (void)hipStreamSynchronize(hipStreamPerThread);
        hip_stub_stall(hipStreamPerThread, 300);
        call(0);
        stage = 1;
        while (stage.load() != 2) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        (void)hipStreamSynchronize(hipStreamPerThread);
    });
    std::thread b([&] {
        while (stage.load() != 1) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        for (int i = 1; i < 13; i++) {
            call(i);
            (void)hipStreamSynchronize(hipStreamPerThread);
        }
        stage = 2;
    });
    a.join();
    b.join();
    for (int i = 0; i < 13; i++) {
        std::vector<uint8_t*> in(K), out(M);
        for (int j = 0; j < K; j++) in[j] = host.data() + (size_t)j * B;
        for (int p = 0; p < M; p++) out[p] = d + (size_t)(K + M * i + p) * B;
        expect_encode(mats[i], K, M, in, out, B, "per-thread scenario");
    }
    const long h = hip_stub_hazards() - before;
    CHECK(h == 0, "per-thread scenario: %ld device-time hazards (a set noted on thread A's per-thread stream was "
                  "covered on thread B's)", h);
    printf("per-thread scenario: %ld device-time hazards\n", h);
    ecg_program_sets_reclaim();
    (void)hipFree(d);
    ecg_set_option(ECG_OPT_PROGRAM_CACHE, 4);
}

}  // namespace

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 8;
    const int ops = argc > 2 ? atoi(argv[2]) : 150;
    const unsigned long long seed = argc > 3 ? strtoull(argv[3], nullptr, 10) : 1;
    std::mt19937_64 rng(seed);
    for (int i = 0; i < 24; i++) {
        std::vector<int> m(K * M);
        for (int& c : m) c = 2 + (int)(rng() % 254);  // never 0 or 1: every program is GENERAL
        g_mats.push_back(m);
    }
    ecg_set_option(ECG_OPT_PROGRAM_CACHE, 4);
    ecg_set_option(ECG_OPT_GRAVEYARD, 6);
    {  // the oracle's lazily built field tables, before any thread uses them (test infrastructure)
        int* m = orc_reed_sol_vandermonde_coding_matrix(2, 2);
        uint8_t a[16] = {1}, b[16] = {2}, c[32];
        uint8_t* in[2] = {a, b};
        uint8_t* out[2] = {c, c + 16};
        orc_matrix_encode(2, 2, m, in, out, 16);
        orc_free(m);
    }
    per_thread_scenario();
    for (auto& d : g_doing) d = "starting";
    std::atomic<bool> finished{false};
    std::thread watchdog([&] {  // a hang names what every thread was doing, then the run fails
        for (int i = 0; i < 600 && !finished; i++) std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (finished) return;
        for (int t = 0; t < T; t++) fprintf(stderr, "watchdog: thread %d stuck in %s\n", t, g_doing[t & 63].load());
        fflush(stderr);
        _exit(3);
    });
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back([t, ops, seed] { Worker(t, seed).run(ops); });
    for (auto& x : th) x.join();
    finished = true;
    watchdog.join();
    int left = 0;
    for (int d = 0; d < kDev; d++) {
        ecg_set_device(d);
        left += ecg_program_sets_reclaim();
    }
    ecg_set_device(0);
    const long hazards = hip_stub_hazards();
    // the run must have exercised the asynchronous paths it is for: queries that found work still pending,
    // and evicted sets waiting for their covers
    printf("coverage: %ld not-ready queries, up to %d evicted sets waiting at once\n", hip_stub_not_ready(),
           g_max_retiring.load());
    const bool covered = hip_stub_not_ready() > 0 && g_max_retiring.load() > 0;
    printf("engine race done: %d threads x %d ops, %ld checks, %d failed, %ld device-time hazards, %d sets left after "
           "reclaim%s\n", T, ops, g_checks.load(), g_fail.load(), hazards, left, covered ? "" : ", PATHS NOT EXERCISED");
    return g_fail.load() == 0 && hazards == 0 && left == 0 && covered ? 0 : 1;
}
