// Config 3's partial-decoding repair as the reference issues it -- per stripe, a helper proxy's partial
// decode, the main proxy's partial decode, then perform_addition of the two (handle_repair.cpp:249,
// 371-376) -- through the C ABI on HBM blocks, in four forms:
//   direct   each call launched on its own (no scope);
//   scope    the same calls inside deferred-batch scopes (one launch per plan per scope);
//   scratch  the same calls, scopes with the partial buffers declared scratch (ecg_batch_scratch): the
//            three calls of a repair compose into one region product, the partials are never written;
//   fused    one encode_partial_blocks_for_decoding over all survivors per repair, in scopes (the
//            single-launch form the scratch composition should match).
// Azure-LRC(12,2,2), local repairs (block e = local[s mod 14] of stripe s), S stripes of 16 blocks.
// Every form is checked against the lost blocks.  Prints one JSON line per form.
// Build: hipcc -O2 -std=c++20 --offload-arch=gfx950 -Iinclude profiles/r02/scope_repair/scope_repair.cpp -Lerasure-codes-prototype_amd/lib
//        -lecg -Wl,-rpath,'$ORIGIN/../erasure-codes-prototype_amd/lib' -o profiles/r02/scope_repair/scope_repair
// Run:   profiles/r02/scope_repair/scope_repair [B_bytes] [S] [steps] [chunk_stripes]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

struct Repair {
    int e;
    std::vector<int> surv, helper, main_;
};

// Local repair of block e of Azure-LRC(12,2,2) under the OPTIMAL partition {0,1,2},{3,4,5},{6,7,8},
// {9,10,11},{14,15,12,13} (bench.py azure_local_split): the group's 6
// survivors, split into the helper partition's survivors and the main proxy's own + direct blocks.
static Repair local_repair(int e) {
    static const std::vector<std::vector<int>> parts = {{0, 1, 2}, {3, 4, 5}, {6, 7, 8}, {9, 10, 11}, {14, 15, 12, 13}};
    Repair r;
    r.e = e;
    const int gid = e < 12 ? e / 6 : e - 14;
    for (int b = 6 * gid; b < 6 * gid + 6; b++)
        if (b != e) r.surv.push_back(b);
    if (14 + gid != e) r.surv.push_back(14 + gid);
    const std::vector<int>* mine = nullptr;
    for (auto& p : parts)
        if (std::count(p.begin(), p.end(), e)) mine = &p;
    std::vector<int> own;
    std::vector<std::vector<int>> sets;  // helper partitions' survivors, then the main proxy's own
    for (int b : r.surv)
        if (std::count(mine->begin(), mine->end(), b)) own.push_back(b);
    for (auto& p : parts) {
        if (&p == mine) continue;
        std::vector<int> in;
        for (int b : r.surv)
            if (std::count(p.begin(), p.end(), b)) in.push_back(b);
        if (in.size() > 1) sets.push_back(in);  // a helper sends one partial (handle_repair.cpp:169-176)
        else own.insert(own.end(), in.begin(), in.end());
    }
    if (!own.empty()) sets.push_back(own);
    if (sets.size() != 2) {
        fprintf(stderr, "unexpected split for block %d\n", e);
        exit(1);
    }
    r.helper = sets[0];
    r.main_ = sets[1];
    return r;
}

int main(int argc, char** argv) {
    const long long B = argc > 1 ? atoll(argv[1]) : (1LL << 20);
    const int S = argc > 2 ? atoi(argv[2]) : 4096;
    const int steps = argc > 3 ? atoi(argv[3]) : 5;
    const int chunk = argc > 4 ? atoi(argv[4]) : 512;
    const int n = 16;
    ecg_coding_parameters cp{};
    cp.k = 12;
    cp.l = 2;
    cp.g = 2;
    cp.local_or_column = 1;
    ecg_ec* ec = ecg_ec_factory(ECG_AZURE_LRC, &cp);
    OK(ecg_ec_init_coding_parameters(ec, &cp));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    OK(ecg_ec_set_memory(ec, ECG_MEM_DEVICE, st));
    uint8_t *stripes, *partials, *out;
    CK(hipMalloc(&stripes, (size_t)S * n * B));
    CK(hipMalloc(&partials, (size_t)S * 2 * B));
    CK(hipMalloc(&out, (size_t)S * B));
    OK(ecg_fill_random(stripes, (long long)S * n * B, 0x5C0DE, 0, st));
    std::vector<int> M(4 * 12);
    OK(ecg_ec_make_encoding_matrix(ec, M.data()));
    OK(ecg_encode_batch(12, 4, M.data(), stripes, n * B, B, stripes + 12 * B, n * B, B, B, S, st));
    const int local[14] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 14, 15};
    std::vector<Repair> plan(S);
    for (int s = 0; s < S; s++) plan[s] = local_repair(local[s % 14]);
    auto blk = [&](int s, int b) { return (char*)(stripes + ((size_t)s * n + b) * B); };
    auto part = [&](int s, int i) { return (char*)(partials + ((size_t)s * 2 + i) * B); };
    auto outp = [&](int s) { return (char*)(out + (size_t)s * B); };
    auto repair_seq = [&](int s) {
        const Repair& r = plan[s];
        char* pp[2] = {part(s, 0), part(s, 1)};
        const std::vector<int>* sets[2] = {&r.helper, &r.main_};
        for (int i = 0; i < 2; i++) {
            std::vector<char*> d;
            for (int b : *sets[i]) d.push_back(blk(s, b));
            OK(ecg_ec_encode_partial_blocks_for_decoding(ec, d.data(), &pp[i], (int)B, sets[i]->data(), (int)sets[i]->size(),
                                                         r.surv.data(), (int)r.surv.size(), &r.e, 1));
        }
        char* o = outp(s);
        OK(ecg_ec_perform_addition(ec, pp, &o, (int)B, 2, 1));
    };
    auto repair_fused = [&](int s) {
        const Repair& r = plan[s];
        std::vector<char*> d;
        for (int b : r.surv) d.push_back(blk(s, b));
        char* o = outp(s);
        OK(ecg_ec_encode_partial_blocks_for_decoding(ec, d.data(), &o, (int)B, r.surv.data(), (int)r.surv.size(),
                                                     r.surv.data(), (int)r.surv.size(), &r.e, 1));
    };
    // check: out[s] == lost block, on the first 28 stripes (every pattern twice) and the last
    std::vector<uint8_t> h_out(B), h_want(B);
    auto check = [&](const char* name) {
        CK(hipStreamSynchronize(st));
        for (int s = 0; s < std::min(S, 28); s++) {
            CK(hipMemcpy(h_out.data(), outp(s), B, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h_want.data(), blk(s, plan[s].e), B, hipMemcpyDeviceToHost));
            if (memcmp(h_out.data(), h_want.data(), B)) {
                fprintf(stderr, "%s: stripe %d repaired block differs\n", name, s);
                exit(1);
            }
        }
        const int last = S - 1;
        CK(hipMemcpy(h_out.data(), outp(last), B, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h_want.data(), blk(last, plan[last].e), B, hipMemcpyDeviceToHost));
        if (memcmp(h_out.data(), h_want.data(), B)) {
            fprintf(stderr, "%s: stripe %d repaired block differs\n", name, last);
            exit(1);
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const std::string mode : {"direct", "scope", "scratch", "fused"}) {
        auto one_step = [&]() {
            for (int c0 = 0; c0 < S; c0 += chunk) {
                const int c1 = std::min(S, c0 + chunk);
                const bool scoped = mode != "direct";
                if (scoped) OK(ecg_batch_begin());
                if (mode == "scratch") OK(ecg_batch_scratch(part(c0, 0), (size_t)(c1 - c0) * 2 * B));
                for (int s = c0; s < c1; s++) {
                    if (mode == "fused") repair_fused(s);
                    else repair_seq(s);
                }
                if (scoped) OK(ecg_batch_end());
            }
        };
        CK(hipMemsetAsync(out, 0, (size_t)S * B, st));
        one_step();  // warm-up (plans, program tables, pointer-table slots)
        check(mode.c_str());
        long long rec = 0, comp = 0, launches = 0, mat = 0;
        OK(ecg_batch_last_stats(&rec, &comp, &launches, &mat));
        CK(hipStreamSynchronize(st));
        const double t0 = now();
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < steps; i++) one_step();
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
        const double wall = (now() - t0) / steps;
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double alg = (double)S * 7 * B;  // (survivors + 1) * B per local repair
        printf("{\"form\": \"%s\", \"B\": %lld, \"stripes\": %d, \"chunk_stripes\": %d, \"repairs_per_s\": %.0f, "
               "\"ms_per_batch\": %.3f, \"algorithmic_GBps\": %.1f, \"algorithmic_frac\": %.4f, "
               "\"last_flush\": {\"recorded\": %lld, \"composed\": %lld, \"launches\": %lld, \"materialised\": %lld}}\n",
               mode.c_str(), B, S, chunk, S / wall, wall * 1e3, alg / wall / 1e9, alg / wall / 8e12, rec, comp, launches, mat);
        fflush(stdout);
    }
    CK(hipFree(stripes));
    CK(hipFree(partials));
    CK(hipFree(out));
    ecg_ec_destroy(ec);
    return 0;
}
