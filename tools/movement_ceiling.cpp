// Movement ceiling of the product kernel's own access path.
//
// Runs gf_vec_kernel through the library's own launch_gf (same 128-thread / 2 KiB chunking, NT loads and
// stores, auto XCD grid map) at the headline size, RS(10,4)-shaped, S = 4096 stripes of 1 MiB blocks in one
// [S][15][B] arena (the stripes, then a rebuild block per stripe, as bench.py lays them out):
//   enc_general  10 -> 4 GENERAL, the RS(10,4) Vandermonde matrix, outputs in the stripes   (the headline encode)
//   enc_zero     10 -> 4 BINARY, every mask 0: the same loads, folds and stores, the multiply removed
//   enc_ones     10 -> 4 BINARY, every mask ~0 (XOR parity)
//   dec_general  10 -> 1 GENERAL (parity row 1 re-encoded) into the rebuild blocks          (decode pattern)
//   dec_zero     10 -> 1 BINARY, masks 0, into the rebuild blocks
//   copy_zero     1 -> 1 BINARY, mask 0, into the rebuild blocks
// Fractions are algorithmic bytes ((inputs + outputs) * B per stripe) / HIP-event kernel time / 8 TB/s.
// Cases are interleaved over rounds so clock and placement drift hit them alike.
// Build (after `make -C erasure-codes-prototype_amd`; host-only source, linked with the library's kernel object):
//   hipcc -O2 -std=c++17 -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ierasure-codes-prototype_amd/csrc \
//     -c tools/movement_ceiling.cpp -o /tmp/mc.o
//   hipcc --offload-arch=gfx950 /tmp/mc.o erasure-codes-prototype_amd/build/gf_kernels.o -o tools/movement_ceiling
// Run: tools/movement_ceiling [rounds=3] [reps=10] [stripes=4096] [case-name filter] [maps]
//   maps: the first selected case under grid maps 1 / 2 (G = 1, 16, 64, 128) / 0, interleaved round by round
// Knobs of the launch (read by the library at first use): ECG_GRID_MAP, ECG_MAP_GROUP, ECG_COLS_PER_WG, ECG_NT.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gf_kernels.hpp"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

using ecg::CoefTab;
using ecg::GfLaunch;

// RS(10,4) systematic Vandermonde coding matrix (tests/test_oracle.py pins it)
static const int kRS104[4][10] = {{1, 1, 1, 1, 1, 1, 1, 1, 1, 1},
                                  {1, 147, 138, 73, 93, 161, 103, 58, 99, 178},
                                  {1, 103, 156, 151, 123, 187, 166, 175, 244, 83},
                                  {1, 220, 166, 123, 82, 143, 245, 40, 167, 122}};

struct Case {
    std::string name;
    int k, m;
    bool binary;
    int mask_or_row;  // BINARY: 0 or 1 for every coefficient; GENERAL: -1 = whole RS matrix, r = row r only
    bool to_rebuild;  // outputs into the rebuild blocks (separate region, stride B) instead of the stripes
    CoefTab* d_tabs = nullptr;
    int* d_src = nullptr;
    int* d_dst = nullptr;
    std::vector<double> ms;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int S = argc > 3 ? atoi(argv[3]) : 4096;
    const std::string only = argc > 4 ? argv[4] : "";  // run only the cases whose name contains this
    const long long B = 1LL << 20;
    const int n = 14;
    const size_t stripe_bytes = (size_t)n * B;
    uint8_t* arena = nullptr;
    CK(hipMalloc(&arena, (size_t)S * (n + 1) * B));
    uint8_t* rebuild = arena + (size_t)S * stripe_bytes;
    CK(ecg::launch_fill_splitmix(arena, (long long)S * (n + 1) * B, 0xEC0DE, 0, nullptr));
    CK(hipDeviceSynchronize());

    std::vector<Case> cases = {{"enc_general 10->4", 10, 4, false, -1, false},
                               {"enc_zero    10->4", 10, 4, true, 0, false},
                               {"enc_ones    10->4", 10, 4, true, 1, false},
                               {"dec_general 10->1", 10, 1, false, 1, true},
                               {"dec_zero    10->1", 10, 1, true, 0, true},
                               {"copy_zero    1->1", 1, 1, true, 0, true}};
    if (!only.empty())
        cases.erase(std::remove_if(cases.begin(), cases.end(),
                                   [&](const Case& c) { return c.name.find(only) == std::string::npos; }),
                    cases.end());
    for (Case& c : cases) {
        std::vector<CoefTab> tabs((size_t)c.k * c.m);
        for (int j = 0; j < c.k; j++)
            for (int p = 0; p < c.m; p++) {
                int coef;
                if (c.binary) coef = c.mask_or_row;
                else coef = c.mask_or_row < 0 ? kRS104[p][j] : kRS104[c.mask_or_row][j];
                ecg::make_coef_tab(coef, &tabs[(size_t)j * c.m + p]);
            }
        std::vector<int> src(c.k), dst(c.m);
        for (int j = 0; j < c.k; j++) src[j] = j;
        for (int p = 0; p < c.m; p++) dst[p] = c.to_rebuild ? p : 10 + p;
        CK(hipMalloc(&c.d_tabs, tabs.size() * sizeof(CoefTab)));
        CK(hipMalloc(&c.d_src, src.size() * sizeof(int)));
        CK(hipMalloc(&c.d_dst, dst.size() * sizeof(int)));
        CK(hipMemcpy(c.d_tabs, tabs.data(), tabs.size() * sizeof(CoefTab), hipMemcpyHostToDevice));
        CK(hipMemcpy(c.d_src, src.data(), src.size() * sizeof(int), hipMemcpyHostToDevice));
        CK(hipMemcpy(c.d_dst, dst.data(), dst.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    auto launch = [&](const Case& c) {
        GfLaunch a;
        memset(&a, 0, sizeof(a));
        a.tabs = c.d_tabs;
        a.src_ids = c.d_src;
        a.dst_ids = c.d_dst;
        a.in_base = arena;
        a.in_sstride = (long long)stripe_bytes;
        a.in_bstride = B;
        a.out_base = c.to_rebuild ? rebuild : arena;
        a.out_sstride = c.to_rebuild ? B : (long long)stripe_bytes;
        a.out_bstride = B;
        a.B = B;
        a.k = c.k;
        a.m = c.m;
        a.S = S;
        a.MT = c.m;
        a.rtiles = 1;
        a.binary = c.binary ? 1 : 0;
        CK(ecg::launch_gf(a, ecg::GF_MODE_STRIDED, true, nullptr));
    };
    std::vector<hipEvent_t> ev(reps + 1);
    for (auto& e : ev) CK(hipEventCreate(&e));
    printf("S=%d B=%lld grid_map option=%lld nt=%lld (fraction of 8 TB/s, algorithmic bytes / HIP-event time)\n", S, B,
           ecg::get_option(ECG_OPT_GRID_MAP), ecg::get_option(ECG_OPT_NT));
    // "maps" mode: the first case under each grid-map setting in turn, interleaved round by round in this one
    // process (the settings are library options), so placement and clock drift hit every setting alike
    if (argc > 5 && std::string(argv[5]) == "maps") {
        struct Setting {
            const char* name;
            long long map, group;
            std::vector<double> ms;
        };
        std::vector<Setting> st = {{"map1 (XCD-contiguous)", 1, 1, {}}, {"map2 G=1", 2, 1, {}}, {"map2 G=16", 2, 16, {}},
                                   {"map2 G=64", 2, 64, {}}, {"map2 G=128", 2, 128, {}}, {"map0 (linear)", 0, 1, {}}};
        Case& c = cases.at(0);
        for (int r = 0; r < rounds; r++)
            for (Setting& x : st) {
                ecg::set_option(ECG_OPT_GRID_MAP, x.map);
                ecg::set_option(ECG_OPT_MAP_GROUP, x.group);
                for (int w = 0; w < 2; w++) launch(c);
                CK(hipEventRecord(ev[0], nullptr));
                for (int i = 0; i < reps; i++) {
                    launch(c);
                    CK(hipEventRecord(ev[i + 1], nullptr));
                }
                CK(hipEventSynchronize(ev[reps]));
                for (int i = 0; i < reps; i++) {
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
                    x.ms.push_back(ms);
                }
            }
        const double bytes = (double)S * (c.k + c.m) * B;
        for (Setting& x : st) {
            std::sort(x.ms.begin(), x.ms.end());
            double avg = 0;
            for (double v : x.ms) avg += v;
            avg /= x.ms.size();
            printf("%s | %-22s avg %.4f ms  median %.4f  | frac avg %.4f  median %.4f\n", c.name.c_str(), x.name, avg,
                   x.ms[x.ms.size() / 2], bytes / (avg * 1e-3) / 8e12, bytes / (x.ms[x.ms.size() / 2] * 1e-3) / 8e12);
        }
        return 0;
    }
    for (int r = 0; r < rounds; r++) {
        for (Case& c : cases) {
            for (int w = 0; w < 2; w++) launch(c);
            // back to back, no host wait between launches (clocks drop within tens of ms of idle)
            CK(hipEventRecord(ev[0], nullptr));
            for (int i = 0; i < reps; i++) {
                launch(c);
                CK(hipEventRecord(ev[i + 1], nullptr));
            }
            CK(hipEventSynchronize(ev[reps]));
            for (int i = 0; i < reps; i++) {
                float ms = 0;
                CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
                c.ms.push_back(ms);
            }
        }
        fflush(stdout);
    }
    for (Case& c : cases) {
        std::vector<double> v = c.ms;
        std::sort(v.begin(), v.end());
        double avg = 0;
        for (double x : v) avg += x;
        avg /= v.size();
        const double bytes = (double)S * (c.k + c.m) * B;
        printf("%s  avg %.4f ms  median %.4f  min %.4f  | frac avg %.4f  median %.4f  best %.4f\n", c.name.c_str(), avg,
               v[v.size() / 2], v[0], bytes / (avg * 1e-3) / 8e12, bytes / (v[v.size() / 2] * 1e-3) / 8e12,
               bytes / (v[0] * 1e-3) / 8e12);
    }
    return 0;
}
