// Region-product launches of any k -> m shape in the families layout (one [S][k+m][B] arena, outputs at block ids
// k .. k+m-1 of their own stripe, as the facade's encode writes them), timed with HIP events, under the library's
// launch options (grid map, map group, columns per workgroup), interleaved round by round in one process so clock
// and placement drift hit every setting alike.  Round-6 probe for the families encode rows: does a
// 16 -> 9 BINARY launch (the composed PC(4,1,4,1) encode) lose to 16 -> 8 at the same bytes, and what moves it?
// Build (after `make -C erasure-codes-prototype_amd`):
//   hipcc -O2 -std=c++17 -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ierasure-codes-prototype_amd/csrc \
//     -c tools/shape_probe.cpp -o /tmp/sp.o
//   hipcc --offload-arch=gfx950 /tmp/sp.o erasure-codes-prototype_amd/build/gf_kernels.o -o tools/shape_probe
// Run: tools/shape_probe rounds reps case... ; case = k,m,bin,S[,label] (bin 1 = BINARY, every mask ~0; 0 = GENERAL,
// random non-zero coefficients).  Settings are fixed below; each case runs under each setting every round.
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

struct Setting {
    const char* name;
    long long map, group, cols, nt = 3, pad = -1;
};

struct Case {
    int k, m, bin, S;
    std::string label;
    uint8_t* arena = nullptr;
    CoefTab* tabs = nullptr;
    int* src = nullptr;
    int* dst = nullptr;
    uint8_t** ptrs = nullptr;  // SHAPE_PROBE_MODE=ptrs: [S][k] input then [S][m] output pointers
    int* prog_of = nullptr;    // SHAPE_PROBE_PROGS=N: N coefficient matrices, stripe s runs prog_of[s]
    std::vector<std::vector<double>> ms;  // per setting
};

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: shape_probe rounds reps k,m,bin,S[,label]...\n");
        return 2;
    }
    const int rounds = atoi(argv[1]), reps = atoi(argv[2]);
    const long long B = 1LL << 20;
    // SHAPE_PROBE_SET=maps: grid maps only (the auto rule's choice for outputs in the stripes is map 1);
    // SHAPE_PROBE_SET=nt: the non-temporal policies under the auto map; SHAPE_PROBE_SET=auto: the auto rule only;
    // SHAPE_PROBE_SET=pads: LDS pads (workgroups per CU).  SHAPE_PROBE_MODE=ptrs: pointer-table launches.
    const char* set = getenv("SHAPE_PROBE_SET");
    const std::vector<Setting> st =
        set && std::string(set) == "auto"
            ? std::vector<Setting>{{"auto", 3, 1, 0}}
        : set && std::string(set) == "pads"  // ECG_OPT_MT1_LDS_PAD (2-output launches too in ECG_TUNE_PAD_MT2 builds)
            ? std::vector<Setting>{{"pad 0", 3, 1, 0, 3, 0},          {"pad 16K", 3, 1, 0, 3, 16384},
                                   {"pad 20K", 3, 1, 0, 3, 20480},    {"pad 24K", 3, 1, 0, 3, 24576},
                                   {"pad 28K", 3, 1, 0, 3, 28672}}
        : set && std::string(set) == "maps"
            ? std::vector<Setting>{{"map1", 1, 1, 0}, {"map2 G=1", 2, 1, 0}, {"map2 G=2", 2, 2, 0}, {"map0", 0, 1, 0}}
        : set && std::string(set) == "nt"  // non-temporal policy: bit 0 loads, bit 1 stores (MT <= 8 only)
            ? std::vector<Setting>{{"nt3", 3, 1, 0, 3}, {"nt1 (temporal stores)", 3, 1, 0, 1},
                                   {"nt2 (temporal loads)", 3, 1, 0, 2}, {"nt0", 3, 1, 0, 0}}
            : std::vector<Setting>{{"auto", 3, 1, 0},        {"map0", 0, 1, 0},       {"map2 G=1", 2, 1, 0},
                                   {"map2 G=8", 2, 8, 0},    {"auto 4KiB", 3, 1, 256}, {"auto 8KiB", 3, 1, 512}};
    std::vector<Case> cs;
    for (int i = 3; i < argc; i++) {
        Case c;
        char lab[64] = {0};
        const int n = sscanf(argv[i], "%d,%d,%d,%d,%63s", &c.k, &c.m, &c.bin, &c.S, lab);
        if (n < 4 || c.k < 1 || c.m < 1 || c.S < 8 || c.k > 64 || c.m > (c.bin ? ecg::kMaxMTBin : ecg::kMaxMT)) {
            fprintf(stderr, "bad case %s\n", argv[i]);
            return 2;
        }
        c.label = n == 5 ? lab : argv[i];
        cs.push_back(c);
    }
    unsigned rng = 12345;
    for (Case& c : cs) {
        const size_t bytes = (size_t)c.S * (c.k + c.m) * B;
        // SHAPE_PROBE_ALLOC=contig: physically contiguous arenas (hipDeviceMallocContiguous)
        const char* al = getenv("SHAPE_PROBE_ALLOC");
        if (al && std::string(al) == "contig") CK(hipExtMallocWithFlags((void**)&c.arena, bytes, hipDeviceMallocContiguous));
        else CK(hipMalloc(&c.arena, bytes));
        CK(ecg::launch_fill_splitmix(c.arena, (long long)bytes, 0xEC0DE, 0, nullptr));
        // SHAPE_PROBE_PROGS=N[,sorted]: N programs (the matrices of a scope's per-pattern repairs), dealt to the
        // stripes round robin (s % N, as per-stripe patterns arrive) or sorted (runs of S / N stripes)
        const char* pe = getenv("SHAPE_PROBE_PROGS");
        const int nprog = pe ? std::max(1, atoi(pe)) : 1;
        const bool sorted = pe && strstr(pe, "sorted");
        std::vector<CoefTab> tabs((size_t)nprog * c.k * c.m);
        for (int q = 0; q < nprog; q++)
            for (int j = 0; j < c.k; j++)
                for (int p = 0; p < c.m; p++) {
                    rng = rng * 1103515245u + 12345u;
                    ecg::make_coef_tab(c.bin ? 1 : 1 + (int)((rng >> 16) % 255), &tabs[((size_t)q * c.k + j) * c.m + p]);
                }
        if (nprog > 1) {
            std::vector<int> po(c.S);
            for (int s_ = 0; s_ < c.S; s_++) po[s_] = sorted ? (int)((long long)s_ * nprog / c.S) : s_ % nprog;
            CK(hipMalloc(&c.prog_of, po.size() * sizeof(int)));
            CK(hipMemcpy(c.prog_of, po.data(), po.size() * sizeof(int), hipMemcpyHostToDevice));
        }
        std::vector<int> src(c.k), dst(c.m);
        for (int j = 0; j < c.k; j++) src[j] = j;
        for (int p = 0; p < c.m; p++) dst[p] = c.k + p;
        CK(hipMalloc(&c.tabs, tabs.size() * sizeof(CoefTab)));
        CK(hipMalloc(&c.src, src.size() * sizeof(int)));
        CK(hipMalloc(&c.dst, dst.size() * sizeof(int)));
        CK(hipMemcpy(c.tabs, tabs.data(), tabs.size() * sizeof(CoefTab), hipMemcpyHostToDevice));
        CK(hipMemcpy(c.src, src.data(), src.size() * sizeof(int), hipMemcpyHostToDevice));
        CK(hipMemcpy(c.dst, dst.data(), dst.size() * sizeof(int), hipMemcpyHostToDevice));
        std::vector<uint8_t*> pt((size_t)c.S * (c.k + c.m));
        for (int s_ = 0; s_ < c.S; s_++) {
            uint8_t* base = c.arena + (size_t)s_ * (c.k + c.m) * B;
            for (int j = 0; j < c.k; j++) pt[(size_t)s_ * c.k + j] = base + (size_t)j * B;
            for (int p = 0; p < c.m; p++) pt[(size_t)c.S * c.k + (size_t)s_ * c.m + p] = base + (size_t)(c.k + p) * B;
        }
        CK(hipMalloc(&c.ptrs, pt.size() * sizeof(uint8_t*)));
        CK(hipMemcpy(c.ptrs, pt.data(), pt.size() * sizeof(uint8_t*), hipMemcpyHostToDevice));
        c.ms.resize(st.size());
    }
    CK(hipDeviceSynchronize());
    const char* md = getenv("SHAPE_PROBE_MODE");
    const bool ptrs_mode = md && std::string(md) == "ptrs";
    printf("mode %s\n", ptrs_mode ? "PTRS (pointer tables, outputs apart)" : "STRIDED");
    auto launch = [&](const Case& c) {
        GfLaunch a;
        memset(&a, 0, sizeof(a));
        a.tabs = c.tabs;
        a.src_ids = c.src;
        a.dst_ids = c.dst;
        a.in_base = c.arena;
        a.out_base = c.arena;
        a.in_sstride = a.out_sstride = (long long)(c.k + c.m) * B;
        a.in_bstride = a.out_bstride = B;
        a.B = B;
        a.k = c.k;
        a.m = c.m;
        a.S = c.S;
        a.MT = c.m;
        a.rtiles = 1;
        a.binary = c.bin;
        a.prog_of_stripe = c.prog_of;
        if (ptrs_mode) {  // as the engine issues a batch scope's repairs: outputs apart from the inputs -> grid map 2
            a.src_ptrs = (const uint8_t* const*)c.ptrs;
            a.dst_ptrs = (uint8_t* const*)(c.ptrs + (size_t)c.S * c.k);
            a.grid_map = 2;
            CK(ecg::launch_gf(a, ecg::GF_MODE_PTRS, true, nullptr));
        } else {
            CK(ecg::launch_gf(a, ecg::GF_MODE_STRIDED, true, nullptr));
        }
    };
    std::vector<hipEvent_t> ev(reps + 1);
    for (auto& e : ev) CK(hipEventCreate(&e));
    for (int r = 0; r < rounds; r++) {
        for (Case& c : cs)
            for (size_t si = 0; si < st.size(); si++) {
                ecg::set_option(ECG_OPT_GRID_MAP, st[si].map);
                ecg::set_option(ECG_OPT_MAP_GROUP, st[si].group);
                ecg::set_option(ECG_OPT_COLS_PER_WG, st[si].cols);
                ecg::set_option(ECG_OPT_NT, st[si].nt);
                ecg::set_option(ECG_OPT_MT1_LDS_PAD, st[si].pad);
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
                    c.ms[si].push_back(ms);
                }
            }
        printf("round %d done\n", r);
        fflush(stdout);
    }
    printf("B=1MiB; frac = (k+m)*B*S / HIP-event time / 8 TB/s; median over %d rounds x %d launches\n", rounds, reps);
    for (Case& c : cs) {
        const double bytes = (double)c.S * (c.k + c.m) * B;
        printf("%-14s k=%2d m=%2d %s S=%4d (%.2f GiB):", c.label.c_str(), c.k, c.m, c.bin ? "BIN" : "GEN", c.S,
               bytes / (1 << 30));
        for (size_t si = 0; si < st.size(); si++) {
            std::vector<double> v = c.ms[si];
            std::sort(v.begin(), v.end());
            printf("  %s %.4f", st[si].name, bytes / (v[v.size() / 2] * 1e-3) / 8e12);
        }
        printf("\n");
    }
    return 0;
}
