// GF(2^8) region-product kernels for MI355X (gfx950, CDNA4).
//
// out_p[x] = XOR_j c[p][j] * in_j[x] over GF(2^8)/0x11d, for p < m, j < k, every byte x of a block.
//
// Data path (HBM-bound, no MFMA -- byte-field XOR-multiply, not a dense contraction):
//   * each lane owns one 16-byte column of every block: one global_load_dwordx4 per input block,
//     64 lanes = 1 KiB contiguous per wave-instruction;
//   * m_out accumulators of 16 bytes stay in VGPRs, so every input byte is read from HBM once and
//     every output byte written once ((k + m) * B bytes per stripe: the algorithmic minimum);
//   * the multiply is three v_perm_b32 table lookups per dword (bit fields [2:0], [5:3], [7:6]) with
//     the per-coefficient tables in SGPRs (scalar loads of a 32-byte CoefTab), folded with gfx950's
//     v_bitop3_b32 (3-input XOR); the bit-field split of an input dword is shared by all m outputs;
//   * straight-line code (no per-coefficient branches); matrices whose entries are all 0/1
//     (perform_addition, LRC local rows, PC merges) take a BINARY flavour: one v_bitop3
//     acc ^ (x & mask) per coefficient-dword.
//   * grid: one kThreads = 128-thread workgroup (2 waves) per 2 KiB chunk of every block of a stripe
//     (cols_per_wg = kThreads 16-byte columns), the workgroup -> chunk map chosen per launch (grid_map
//     auto: XCD-contiguous when the outputs live in the input stripes, stripe-per-XCD otherwise),
//     non-temporal loads and stores -- measured best on MI355X (profiles/r01/microbench.*: 16 KiB chunks
//     5.35 TB/s -> 4 KiB 5.80 -> XCD map 6.14 -> 128 threads / 2 KiB + auto map 6.28-6.33 TB/s).
// VALU cost per 16-byte column: 20 ops to split one input, ~18 per coefficient (GENERAL) or 4
// (BINARY); for RS(10,4) encode ~1000 ops per 160 data bytes, ~35 % of gfx950's integer issue rate
// at the HBM roofline.
#include <atomic>

#include "gf_kernels.hpp"
#include "gf256.hpp"

// gfx950 only: the completion-flag epilogue (gf_done_flag.hpp) encodes its waits for gfx9's vmcnt, which
// counts stores there; gfx10+ count stores in vscnt, and the flag could then overtake the data.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "gf_kernels.hip is gfx950 (CDNA4) code"
#endif

#include "gf_done_flag.hpp"

namespace ecg {

namespace {

// Uniform metadata (coefficient tables, block ids, pointer tables) is read through the constant
// address space so the backend selects scalar (SMEM) loads into SGPRs; through a plain global
// pointer it cannot prove the output stores never clobber it and falls back to per-lane loads.
#define ECG_CONST __attribute__((address_space(4)))
template <typename T>
__device__ __forceinline__ const ECG_CONST T* cst(const T* p) {
    return (const ECG_CONST T*)p;
}

template <int MODE>
__device__ __forceinline__ const uint8_t* src_ptr(const GfLaunch& a, int s, int prog, int j) {
    if constexpr (MODE == GF_MODE_INLINE || MODE == GF_MODE_INLINE_LAT) {
        return a.isrc[j];
    } else if constexpr (MODE == GF_MODE_PTRS) {
        return cst(a.src_ptrs)[(size_t)s * a.k + j];
    } else {
        const long long sa = a.stripe_of ? (long long)cst(a.stripe_of)[s] : (long long)s;
        return a.in_base + sa * a.in_sstride + (long long)cst(a.src_ids)[prog * a.k + j] * a.in_bstride;
    }
}

template <int MODE>
__device__ __forceinline__ uint8_t* dst_ptr(const GfLaunch& a, int s, int prog, int p) {
    if constexpr (MODE == GF_MODE_INLINE || MODE == GF_MODE_INLINE_LAT) {
        return a.idst[p];
    } else if constexpr (MODE == GF_MODE_PTRS) {
        return cst(a.dst_ptrs)[(size_t)s * a.m + p];
    } else {
        const long long sa = a.stripe_of ? (long long)cst(a.stripe_of)[s] : (long long)s;
        return a.out_base + sa * a.out_sstride + (long long)cst(a.dst_ids)[prog * a.m + p] * a.out_bstride;
    }
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// gfx950 v_bitop3_b32, LUT index = S0<<2 | S1<<1 | S2.  0x96 = a ^ b ^ c.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// NT policy bits: 1 = non-temporal loads, 2 = non-temporal stores.
template <int NT>
__device__ __forceinline__ void load16(const uint8_t* p, uint32_t (&x)[4]) {
    u32x4 v;
    if constexpr (NT & 1) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else v = *reinterpret_cast<const u32x4*>(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
}

template <int NT>
__device__ __forceinline__ void store16(uint8_t* p, const uint32_t (&x)[4]) {
    u32x4 v;
    v.x = x[0]; v.y = x[1]; v.z = x[2]; v.w = x[3];
    if constexpr (NT & 2) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else *reinterpret_cast<u32x4*>(p) = v;
}

// Bit-field split of one input dword: the v_perm selectors shared by every output row.
struct Split {
    uint32_t i0, i1, i2;
};

__device__ __forceinline__ Split split(uint32_t x) {
    return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// c * x for the four bytes of one dword: three v_perm lookups + one v_bitop3.
__device__ __forceinline__ uint32_t gmul(const ECG_CONST CoefTab& t, const Split& s) {
    return xor3(perm(t.t0hi, t.t0lo, s.i0), perm(t.t1hi, t.t1lo, s.i1), perm(t.t2, t.t2, s.i2));
}

// GENERAL flavour: U inputs folded into MT accumulators, input pairs share one v_bitop3.  Every
// coefficient goes through the tables (c = 0 and c = 1 tables are exact).
template <int MT, int U>
__device__ __forceinline__ void fold_general(const uint32_t (&x)[U][4], const ECG_CONST CoefTab* t,
                                             uint32_t (&acc)[MT][4]) {
#pragma unroll
    for (int u = 0; u + 1 < U; u += 2) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const Split s0 = split(x[u][d]);
            const Split s1 = split(x[u + 1][d]);
#pragma unroll
            for (int p = 0; p < MT; ++p)
                acc[p][d] = xor3(acc[p][d], gmul(t[u * MT + p], s0), gmul(t[(u + 1) * MT + p], s1));
        }
    }
    if constexpr (U & 1) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const Split s0 = split(x[U - 1][d]);
#pragma unroll
            for (int p = 0; p < MT; ++p) acc[p][d] ^= gmul(t[(U - 1) * MT + p], s0);
        }
    }
}

// BINARY flavour (every coefficient 0 or 1: perform_addition, LRC local rows, PC merges):
// acc ^= x & mask in one v_bitop3 (0x78 = S0 ^ (S1 & S2)), mask = 0 or ~0 from SGPRs.
template <int MT, int U>
__device__ __forceinline__ void fold_binary(const uint32_t (&x)[U][4], const ECG_CONST CoefTab* t,
                                            uint32_t (&acc)[MT][4]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int p = 0; p < MT; ++p) {
            const uint32_t msk = t[u * MT + p].mask;
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[p][d] = __builtin_amdgcn_bitop3_b32(acc[p][d], x[u][d], msk, 0x78);
        }
}

template <int MT, int U, bool BIN>
__device__ __forceinline__ void fold(const uint32_t (&x)[U][4], const ECG_CONST CoefTab* t, uint32_t (&acc)[MT][4]) {
    if constexpr (BIN) fold_binary<MT, U>(x, t, acc);
    else fold_general<MT, U>(x, t, acc);
}

// Minimum waves per EU the register allocator must allow (r01 sweep, tools/gpu_variants.sh): 8 for the
// 1-2-output kernels (decode, repair, XOR: +2 % at 8 vs 6), 6 for 3-4 outputs (encode: 8 costs 1 %),
// 4 above -- except 5 outputs: under the 128-VGPR cap of 4 waves the allocator spilled 12 bytes per lane
// in the GENERAL flavour, while a hint of 3 lets it settle at 82 VGPRs (5 waves) with no scratch (r01; with
// two inputs per load batch since r06 it takes 61, 7 waves).
// ECG_OCC_OVERRIDE is for tuning builds only.
constexpr int occupancy_for(int MT) {
#ifdef ECG_OCC_OVERRIDE
    return MT <= 4 ? ECG_OCC_OVERRIDE : 4;
#else
    return MT <= 2 ? 8 : MT <= 4 ? 6 : MT == 5 ? 3 : 4;  // MT 9-16 (BINARY only): 64 accumulator VGPRs at 16
#endif
}

// Workgroup -> (stripe, column chunk).  grid_map 0: linear (workgroup b takes chunk b).  grid_map 1:
// XCD-contiguous -- the dispatcher deals workgroups round-robin over the 8 XCDs, so b % 8 names the
// XCD group; each group is given a contiguous 1/8 of the chunk list (T1 in the HIP guide; here for
// DRAM locality of the concurrently active chunks, not L2 reuse).  grid_map 2: runs of G = map_group
// adjacent launch stripes are dealt round-robin to the XCD groups (G = 1: stripe s on group s % 8), each
// group takes its stripes and their chunks in order.  Speed only, never correctness.
__device__ __forceinline__ void wg_coords(const GfLaunch& a, int& s, int& w) {
    long long b = blockIdx.x;
    if (a.grid_map == 1) {
        const long long G = (long long)gridDim.x;
        const long long per = G >> 3;  // G % 8 == 0 is checked by the host
        b = (b & 7) * per + (b >> 3);
    } else if (a.grid_map == 2) {  // runs of G stripes dealt to the XCD groups (S % (8 G) == 0 checked by the host)
        const long long i = b >> 3;                  // the i-th workgroup dealt to this XCD group
        const long long ls = i / a.wg_per_stripe;    // the group's ls-th stripe, chunks in order
        const long long G = a.map_group;
        s = (int)(((ls / G) * 8 + (b & 7)) * G + ls % G);
        w = (int)(i - ls * a.wg_per_stripe);
        return;
    }
    s = (int)(b / a.wg_per_stripe);
    w = (int)(b - (long long)s * a.wg_per_stripe);
}

// The program of launch stripe s; s becomes the stripe it addresses.  Row split (STRIDED, row_split = R):
// launch stripe s is output row s % R of stripe s / R, run as its own program (the host split each
// program into R single-row programs whose inputs are that row's own, engine.cpp run_strided).
template <int MODE>
__device__ __forceinline__ int launch_prog(const GfLaunch& a, int& s) {
    int r = 0;
    if constexpr (MODE == GF_MODE_STRIDED) {
        if (a.row_split) {
            r = s % a.row_split;
            s = s / a.row_split;
        }
    }
    const int p = a.prog_of_stripe ? cst(a.prog_of_stripe)[s] : 0;
    if constexpr (MODE == GF_MODE_STRIDED) return a.row_split ? p * a.row_split + r : p;
    return p;
}

// ---------------------------------------------------------------------------------------------
// Input blocks whose loads a lane keeps in flight before folding them (ECG_TUNE_LOAD_BATCH: tuning builds only).
#ifdef ECG_TUNE_LOAD_BATCH
constexpr int kLoadBatch = ECG_TUNE_LOAD_BATCH;
#else
constexpr int kLoadBatch = 4;
#endif
// GENERAL tiles of 5+ outputs take two: with four, 4 inputs x MT tables (5 dwords each) outgrow the SGPR file and the
// tile needs 87 VGPRs at MT = 5 (5 waves per SIMD); with two it takes 61 (7 waves), and a 12 -> 5 launch (the
// Azure+1 encode) runs 0.745 of 8 TB/s instead of 0.684-0.694, 12 -> 6 0.70 instead of 0.66, 10 -> 8 0.665 instead
// of 0.61 (profiles/r06/families/shape_probe/sp_glb*.log, two processes each).
#ifdef ECG_TUNE_GEN_WIDE_LB
constexpr int kGenWideLB = ECG_TUNE_GEN_WIDE_LB;
#else
constexpr int kGenWideLB = 2;
#endif
#ifdef ECG_TUNE_GEN_LB
constexpr int kGenLB = ECG_TUNE_GEN_LB;  // GENERAL tiles of 1-4 outputs (tuning builds only)
#else
constexpr int kGenLB = 4;
#endif

// Generic vector path: bytes [0, 16 * floor(B / 16)) of every block; all pointers 16-byte aligned.
// grid.x = S * wg_per_stripe (stripe-major), grid.y = row tiles of MT outputs.
template <int MT, int MODE, int NT, bool BIN>
__global__ void __launch_bounds__(kThreads, MODE == GF_MODE_INLINE_LAT ? 1 : occupancy_for(MT)) gf_vec_kernel(const GfLaunch a) {
    int s, w;
    wg_coords(a, s, w);
    const int rt = blockIdx.y;
    const int prog = launch_prog<MODE>(a, s);
    const int k = a.k;
    const int row0 = rt * MT;
    const int nrows = min(MT, a.m - row0);
    const ECG_CONST CoefTab* T = cst(a.tabs) + (size_t)(prog * a.rtiles + rt) * (size_t)k * MT;
    const long long ncols = a.B >> 4;
    const long long c0 = (long long)w * a.cols_per_wg;
    const long long c1 = min(c0 + (long long)a.cols_per_wg, ncols);

    uint8_t* dst[MT];
#pragma unroll
    for (int p = 0; p < MT; ++p) dst[p] = (p < nrows) ? dst_ptr<MODE>(a, s, prog, row0 + p) : nullptr;

    for (long long c = c0 + threadIdx.x; c < c1; c += kThreads) {
        const long long off = c << 4;
        uint32_t acc[MT][4];
#pragma unroll
        for (int p = 0; p < MT; ++p)
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[p][d] = 0u;

        int j = 0;
        if constexpr (MODE == GF_MODE_INLINE_LAT) {
            // uniform: every load in flight before the first use, then fold.  Straight-line loads (a
            // lane past k re-reads input 0): a branch per load would end the basic block and with it the
            // overlap, one PCIe round trip per input.
            if (k <= 8) {
                uint32_t x[8][4];
#pragma unroll
                for (int u = 0; u < 8; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, u < k ? u : 0) + off, x[u]);
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (u < k) fold<MT, 1, BIN>(reinterpret_cast<const uint32_t(&)[1][4]>(x[u]), T + (size_t)u * MT, acc);
                j = k;
            } else if (k <= 16) {
                uint32_t x[16][4];
#pragma unroll
                for (int u = 0; u < 16; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, u < k ? u : 0) + off, x[u]);
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (u < k) fold<MT, 1, BIN>(reinterpret_cast<const uint32_t(&)[1][4]>(x[u]), T + (size_t)u * MT, acc);
                j = k;
            }
        }
        constexpr int LB = BIN ? kLoadBatch : MT >= 5 ? kGenWideLB : kGenLB;
        for (; j + LB <= k; j += LB) {
            uint32_t x[LB][4];
#pragma unroll
            for (int u = 0; u < LB; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off, x[u]);
            fold<MT, LB, BIN>(x, T + (size_t)j * MT, acc);
        }
        if constexpr (LB > 4) {  // the rest of k: four, two, one
            if (j + 4 <= k) {
                uint32_t x[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off, x[u]);
                fold<MT, 4, BIN>(x, T + (size_t)j * MT, acc);
                j += 4;
            }
        }
        if (j + 2 <= k) {
            uint32_t x[2][4];
#pragma unroll
            for (int u = 0; u < 2; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off, x[u]);
            fold<MT, 2, BIN>(x, T + (size_t)j * MT, acc);
            j += 2;
        }
        if (j < k) {
            uint32_t x[1][4];
            load16<NT>(src_ptr<MODE>(a, s, prog, j) + off, x[0]);
            fold<MT, 1, BIN>(x, T + (size_t)j * MT, acc);
        }
#pragma unroll
        for (int p = 0; p < MT; ++p)
            if (p < nrows) store16<NT>(dst[p] + off, acc[p]);
    }
    if constexpr (MODE == GF_MODE_INLINE_LAT) {
        if (a.done_flags) post_done_flag(a);
    }
}

// Latency kernel for small zero-copy host calls (GF_MODE_INLINE_LAT, blocks <= ECG_OPT_LAT_DWORD_BYTES):
// one DWORD column per lane instead of 16 bytes.  A 1 KiB call is 64 sixteen-byte columns, i.e. ONE wave
// that runs the whole multiply (~550 VALU instructions per lane for RS(6,4)) after its PCIe loads; at 4
// bytes per lane the same bytes are 256 lanes in 4 waves on 4 SIMDs, each with a quarter of the multiply.
// KB = the input count rounded up to a bucket (k <= KB): straight-line code over KB inputs, every input
// load in flight at once.  Padded inputs (u >= k) re-read input 0 with table 0 and are masked out of the sum.
// kLatThreads dword columns per workgroup; grid.x = ceil((B / 4) / kLatThreads), one row tile (m <= kMaxMT).
//
// Coefficient tables through LDS (round 4).  The row tile's k * MT tables are k * MT * 5 dwords: 200 for
// RS(10,4), more than the SGPR file holds, so as scalar loads they came in ~40 dependent rounds of
// s_load + s_waitcnt lgkmcnt(0) (plus SGPR spills to VGPR lanes), each an L2 round trip when a CU's first
// wave runs -- and a single call has about one wave per CU.  A 64 KiB RS(10,4) device call took 5.8 us of
// kernel time for 896 KiB of traffic (profiles/r04/lat_tables/).  Now every wave fetches the tile's tables
// with one to four 16-byte loads per lane, issued BEFORE its data loads (loads return in order, so waiting
// for them does not wait for the data), writes them into its own LDS slice and reads them back, input by
// input, as VGPR operands of v_perm (lat_fold_lds).  A wave reads only its own slice, in program order, so
// no barrier is needed.
template <int MT, int KB>
struct LatTabs {
    static constexpr int kPieces = KB * MT * 2;             // 16-byte pieces of the largest tile of this bucket
    static constexpr int kPerLane = (kPieces + 63) / 64;    // loads per lane
    CoefTab t[kLatThreads / 64][KB * MT];                   // one slice per wave
};

// The latency kernel's own argument block (round 5).  A single call's launch is host-bound: the runtime
// writes the kernel arguments into device-visible memory per launch, and a back-to-back launch costs 2.74 us
// of host time with 24 bytes of arguments against 3.51 us with GfLaunch's 1432 (launch_floor_host_run*.txt,
// profiles/r04/lat_tables/).  LatArgs carries only what the kernel reads -- KB input and MT output pointers
// (80 bytes for config 3's 4 -> 1 bucket, 232 for the largest) -- and takes one row tile (m <= kMaxMT; wider
// single calls run gf_vec_kernel).
template <int KB, int MT>
struct LatArgs {
    const CoefTab* tabs;  // [k][MT]
    unsigned* done_flags;
    long long B;
    int k, m;
    unsigned done_seq;
    const uint8_t* src[KB];  // slots u >= k repeat input 0
    uint8_t* dst[MT];        // slots p >= m repeat output 0 (never stored)
};

template <int MT, int KB>
__device__ __forceinline__ void lat_tabs_load(const LatArgs<KB, MT>& a, u32x4 (&tv)[LatTabs<MT, KB>::kPerLane]) {
    const u32x4* src = reinterpret_cast<const u32x4*>(a.tabs);
    const int last = a.k * MT * 2 - 1;  // this tile's last piece (k <= KB)
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < LatTabs<MT, KB>::kPerLane; ++i) tv[i] = src[min(lane + 64 * i, last)];
}

template <int MT, int KB>
__device__ __forceinline__ const CoefTab* lat_tabs_store(LatTabs<MT, KB>& lds,
                                                         const u32x4 (&tv)[LatTabs<MT, KB>::kPerLane]) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    u32x4* dst = reinterpret_cast<u32x4*>(lds.t[wave]);
#pragma unroll
    for (int i = 0; i < LatTabs<MT, KB>::kPerLane; ++i)
        if (lane + 64 * i < LatTabs<MT, KB>::kPieces) dst[lane + 64 * i] = tv[i];
    return lds.t[wave];
}

// The fold of the latency kernel and the call worker over LDS tables, read just in time: input u + 1's
// tables are read while input u is folded, so at most two inputs' tables are live in VGPRs.  Hoisting all
// of them (what the compiler does otherwise) costs k * MT * 5 VGPRs: 243 VGPRs for RS(10,4) -- two waves
// per SIMD -- and a scratch spill for a 16-input, 8-output tile; read just in time they take 60 and 71
// (tests/test_kernel_resources.py).  The order is pinned by an empty asm per input that consumes the
// accumulators and clobbers memory: input u's folds are done before it, and input u + 2's LDS reads cannot
// move above it (a scheduling barrier does not hold: instruction selection already sinks the arithmetic to
// its last use and hoists the loads).
template <int MT, bool BIN, int KB>
__device__ __forceinline__ void lat_fold_lds(const int k, const CoefTab* T, const uint32_t (&x)[KB],
                                             uint32_t (&acc)[MT]) {
    struct R {
        uint32_t t0lo, t0hi, t1lo, t1hi, t2;
    };
    auto rd = [&](int u, R (&r)[MT]) {
        const CoefTab* t = T + (size_t)(u < k ? u : 0) * MT;
#pragma unroll
        for (int p = 0; p < MT; ++p) {
            if constexpr (BIN) r[p].t0lo = t[p].mask;
            else r[p] = {t[p].t0lo, t[p].t0hi, t[p].t1lo, t[p].t1hi, t[p].t2};
        }
    };
#pragma unroll
    for (int p = 0; p < MT; ++p) acc[p] = 0u;
    R cur[MT], nxt[MT];
    rd(0, cur);
#pragma unroll
    for (int u = 0; u < KB; ++u) {
        if (u + 1 < KB) rd(u + 1, nxt);
        const uint32_t keep = u < k ? ~0u : 0u;  // uniform: padded inputs (u >= k) are masked out
        if constexpr (BIN) {
#pragma unroll
            for (int p = 0; p < MT; ++p) acc[p] = __builtin_amdgcn_bitop3_b32(acc[p], x[u], cur[p].t0lo & keep, 0x78);
        } else {
            const Split sp = split(x[u]);
#pragma unroll
            for (int p = 0; p < MT; ++p) {
                const uint32_t g = xor3(perm(cur[p].t0hi, cur[p].t0lo, sp.i0), perm(cur[p].t1hi, cur[p].t1lo, sp.i1),
                                        perm(cur[p].t2, cur[p].t2, sp.i2));
                acc[p] = __builtin_amdgcn_bitop3_b32(acc[p], g, keep, 0x78);
            }
        }
#pragma unroll
        for (int p = 0; p < MT; ++p) asm volatile("" : "+v"(acc[p]) : : "memory");
        if (u + 1 < KB)
#pragma unroll
            for (int p = 0; p < MT; ++p) cur[p] = nxt[p];
    }
}

// The latency kernel's output stores are non-temporal.  Write-through stores (`sc0 sc1`: the line leaves the
// XCD's L2 with the store, so the end-of-kernel release and the flag epilogue's L2 write-back find nothing
// dirty) were tried for single calls: config 3's per-call sequence A/B over two boxes went 0.119-0.135 ->
// 0.135-0.141 on one and 0.124-0.145 -> 0.123-0.131 on the other, i.e. within the spread
// (profiles/r05/percall_args/latsc1/).  ECG_TUNE_LAT_STORE_SC1 builds them (tuning builds only).
__device__ __forceinline__ void lat_store(uint32_t* p, uint32_t v) {
#ifdef ECG_TUNE_LAT_STORE_SC1
    asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
#else
    __builtin_nontemporal_store(v, p);
#endif
}

// EAGER (blocks <= kLatEagerBytes): a scheduling barrier keeps every input load ahead of the fold.  RS(6,4)
// 1 KiB host calls 0.3-2 us faster (A/B of two builds over two boxes, profiles/r02/lat_kernel/eager/);
// single device calls at 64 KiB - 1 MiB measured 1-5 % slower with it, so only small blocks take it.
// Every lane runs the whole body: lanes past the end load the last column and store nothing, so no branch
// precedes the loads and a wave past the end still reaches the flag epilogue.
template <int MT, bool BIN, int KB, bool EAGER>
__global__ void __launch_bounds__(kLatThreads, 1) gf_lat_dword_kernel(const LatArgs<KB, MT> a) {
    __shared__ LatTabs<MT, KB> lds;
    const int k = a.k;
    const int nrows = a.m;
    const long long ndw = a.B >> 2;
    const long long c = (long long)blockIdx.x * kLatThreads + threadIdx.x;
    // Every pointer slot is read with a constant index (the host filled the padded slots): one round of
    // kernel-argument loads, no address computed from k; the flag word in the same round (not after the fold).
    const uint8_t* src[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) src[u] = a.src[u];
    uint8_t* dst[MT];
#pragma unroll
    for (int p = 0; p < MT; ++p) dst[p] = a.dst[p];
    unsigned* const flags = a.done_flags;
    // the table loads go out first
    u32x4 tv[LatTabs<MT, KB>::kPerLane];
    lat_tabs_load<MT, KB>(a, tv);
    __builtin_amdgcn_sched_barrier(0);
    const bool live = c < ndw;
    const long long off = (live ? c : ndw - 1) << 2;
    uint32_t x[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) x[u] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(src[u] + off));
    if constexpr (EAGER) __builtin_amdgcn_sched_barrier(0);
    const CoefTab* T = lat_tabs_store<MT, KB>(lds, tv);
    uint32_t acc[MT];
    lat_fold_lds<MT, BIN, KB>(k, T, x, acc);
    if (live) {
#pragma unroll
        for (int p = 0; p < MT; ++p)
            if (p < nrows) lat_store(reinterpret_cast<uint32_t*>(dst[p] + off), acc[p]);
    }
    if (flags) post_done_flag(flags + blockIdx.x, a.done_seq);
}

// ---------------------------------------------------------------------------------------------
// Resident call worker (gf_kernels.hpp WorkerArgs; engine.cpp CallWorker).  Workgroup 0 (the leader)
// polls the descriptor ring in pinned host memory and the host's stop word -- one PCIe round trip per
// poll -- and republishes each descriptor it takes in a device-memory mailbox, which the other
// workgroups poll (L2), so an idle worker reads 256 bytes over the link per poll, not 256 per workgroup.
// Each call then runs like gf_lat_dword_kernel (4 bytes per lane, every input load in flight at once,
// KB-bucket straight-line fold) over the workgroup's dword columns, and every workgroup posts its flag
// with the same release sequence (gf_done_flag.hpp); it takes each call's inputs behind a system-scope
// acquire, as a fresh launch would.  Bounded: a workgroup exits on the stop word, on
// the leader's exit word, after idle_ticks without a call or life_ticks in total (followers: twice both,
// as a backstop) or after max_polls polls -- whichever comes first -- and writes `gen` into its
// exit_info slot as it goes, so the host knows when the whole generation is gone.

__device__ __forceinline__ unsigned long long wk_ptr(const unsigned* d, int q) {
    return ((unsigned long long)d[worker_pos(q + 1)] << 32) | d[worker_pos(q)];
}

// The call's tables go through the wave's LDS slice `wt` as in the latency kernel (one to two 16-byte loads
// per lane, issued before the data loads; lat_fold_lds): through SGPRs they spilled 1324 SGPRs to VGPR
// lanes in this kernel.  A generation is at least as wide as its calls (CallWorker: W >= need), so a lane
// has at most one column; the loop after it is a backstop.
template <int MT, bool BIN, int KB>
__device__ __forceinline__ void worker_call(const unsigned* d, CoefTab* wt) {
    const int k = (int)d[worker_pos(WF_K)];
    const int m = (int)d[worker_pos(WF_M)];
    const long long ndw = (long long)d[worker_pos(WF_B)] >> 2;
    const u32x4* tg = reinterpret_cast<const u32x4*>((uintptr_t)wk_ptr(d, WF_TABS));
    const uint8_t* in[KB];
#pragma unroll
    for (int u = 0; u < KB; u++) in[u] = (const uint8_t*)(uintptr_t)wk_ptr(d, WF_IN + 2 * (u < k ? u : 0));
    uint8_t* out[MT];
#pragma unroll
    for (int p = 0; p < MT; p++) out[p] = (uint8_t*)(uintptr_t)wk_ptr(d, WF_OUT + 2 * (p < m ? p : 0));
    constexpr int kPieces = KB * MT * 2, kPerLane = (kPieces + 63) / 64;
    const int last = k * MT * 2 - 1, lane = threadIdx.x & 63;
    u32x4 tv[kPerLane];
#pragma unroll
    for (int i = 0; i < kPerLane; ++i) tv[i] = tg[min(lane + 64 * i, last)];
    __builtin_amdgcn_sched_barrier(0);
    const long long stride = (long long)gridDim.x * kLatThreads;
    long long c = (long long)blockIdx.x * kLatThreads + threadIdx.x;
    const bool live = c < ndw;
    uint32_t x[KB];
#pragma unroll
    for (int u = 0; u < KB; u++) x[u] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(in[u]) + (live ? c : 0));
#pragma unroll
    for (int i = 0; i < kPerLane; ++i)
        if (lane + 64 * i < kPieces) reinterpret_cast<u32x4*>(wt)[lane + 64 * i] = tv[i];
    uint32_t acc[MT];
    lat_fold_lds<MT, BIN, KB>(k, wt, x, acc);
    if (live) {
#pragma unroll
        for (int p = 0; p < MT; p++)
            if (p < m) __builtin_nontemporal_store(acc[p], reinterpret_cast<uint32_t*>(out[p]) + c);
    }
    for (c += stride; c < ndw; c += stride) {
#pragma unroll
        for (int u = 0; u < KB; u++) x[u] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(in[u]) + c);
        lat_fold_lds<MT, BIN, KB>(k, wt, x, acc);
#pragma unroll
        for (int p = 0; p < MT; p++)
            if (p < m) __builtin_nontemporal_store(acc[p], reinterpret_cast<uint32_t*>(out[p]) + c);
    }
}

template <int MT, bool BIN>
__device__ __forceinline__ void worker_call_k(const unsigned* d, CoefTab* wt) {
    const unsigned k = d[worker_pos(WF_K)];
    if (k <= 4) worker_call<MT, BIN, 4>(d, wt);
    else if (k <= 6) worker_call<MT, BIN, 6>(d, wt);
    else if (k <= 8) worker_call<MT, BIN, 8>(d, wt);
    else if (k <= 10) worker_call<MT, BIN, 10>(d, wt);
    else if (k <= 12) worker_call<MT, BIN, 12>(d, wt);
    else worker_call<MT, BIN, 16>(d, wt);
}

template <bool BIN>
__device__ __forceinline__ void worker_call_m(const unsigned* d, CoefTab* wt) {
    switch (d[worker_pos(WF_M)]) {
        case 1: worker_call_k<1, BIN>(d, wt); break;
        case 2: worker_call_k<2, BIN>(d, wt); break;
        case 3: worker_call_k<3, BIN>(d, wt); break;
        default: worker_call_k<4, BIN>(d, wt); break;
    }
}

__global__ void __launch_bounds__(kLatThreads, 1) gf_call_worker_kernel(const WorkerArgs a) {
    __shared__ unsigned d[64];
    __shared__ unsigned go;  // set by thread 0 only: every exit decision is one for the whole workgroup
    __shared__ CoefTab wtabs[kLatThreads / 64][kWorkerMaxSrc * kWorkerMaxRows];  // one table slice per wave
    const int tid = threadIdx.x;
    const bool leader = blockIdx.x == 0;
    unsigned next = a.start_seq;
    const unsigned long long t0 = wall_clock64();
    unsigned long long last = t0;
    // The leader decides when a generation ends: on the stop word, after idle_ticks without a call, and --
    // busy or not -- by not taking a call once life_ticks are over (the host then starts a new generation
    // at that call).  It tells the others through the exit word; their own limits are twice as long, a
    // backstop only: a follower leaving first would strand the calls the leader takes.
    const unsigned long long my_idle = leader ? a.idle_ticks : 2 * a.idle_ticks;
    const unsigned long long my_life = leader ? a.life_ticks : 2 * a.life_ticks;
    for (unsigned polls = 0; polls < a.max_polls; polls++) {
        const unsigned slot = next % (unsigned)kWorkerSlots;
        if (leader) {
            if (tid < 64) {  // wave 0: the descriptor and the stop word in one round trip
                const unsigned v = __hip_atomic_load(&a.ring[slot].w[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const unsigned stop = __hip_atomic_load(a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                d[tid] = v;
                if (tid == 0) go = stop ? 2u : 0u;
            }
            __syncthreads();
            if (tid == 0 && go == 0) {
                const unsigned long long t = wall_clock64();
                if (t - t0 > my_life) go = 2;
                else if (d[0] == next && d[16] == next && d[32] == next && d[48] == next) go = 1;
                else if (t - last > my_idle) go = 2;
            }
            __syncthreads();
            if (go == 1 && gridDim.x > 1 && tid < 64) {  // republish for the followers: payload, then seq
                __hip_atomic_store(&a.mbox[slot].w[tid], d[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tid == 0) __hip_atomic_store(&a.mbseq[slot], next, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            if (tid == 0) {
                const unsigned sq = __hip_atomic_load(&a.mbseq[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned ex = __hip_atomic_load(&a.mbseq[kWorkerSlots], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long t = wall_clock64();
                go = sq == next ? 1u : (ex == a.gen || t - last > my_idle || t - t0 > my_life) ? 2u : 0u;
            }
            __syncthreads();
            if (go == 1 && tid < 64)
                d[tid] = __hip_atomic_load(&a.mbox[slot].w[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
        }
        const unsigned g = go;
        if (g == 2) break;
        if (g == 0) {
            __syncthreads();  // d / go are rewritten by the next poll
            continue;
        }
        // Acquire at system scope before the call's inputs are read: the staging area is reused call after
        // call, and a resident kernel -- unlike a fresh launch, whose start invalidates the caches -- would
        // otherwise read lines of an earlier call's inputs still held in the CU / L2 caches (every call
        // after the first one read stale data without this, tests/test_gpu_worker.py).
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        CoefTab* const wt = wtabs[tid >> 6];
        if (d[worker_pos(WF_BINARY)]) worker_call_m<true>(d, wt);
        else worker_call_m<false>(d, wt);
        post_done_flag(a.flags + (size_t)slot * kWorkerMaxWG + blockIdx.x, next);
        next++;
        last = wall_clock64();
        __syncthreads();
    }
    // No release needed on the way out: nothing follows these stores, and every output of the workgroup
    // went out behind its call's flag.
    if (tid == 0) {
        if (leader) __hip_atomic_store(&a.mbseq[kWorkerSlots], a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.exit_info + blockIdx.x, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Byte path: bytes [off0, B) (tails, unaligned pointers).  cols_per_wg = bytes per workgroup.
template <int MT, int MODE, bool BIN>
__global__ void __launch_bounds__(kThreads) gf_byte_kernel(const GfLaunch a) {
    int s, w;
    wg_coords(a, s, w);
    const int rt = blockIdx.y;
    const int prog = launch_prog<MODE>(a, s);
    const int k = a.k;
    const int row0 = rt * MT;
    const int nrows = min(MT, a.m - row0);
    const ECG_CONST CoefTab* T = cst(a.tabs) + (size_t)(prog * a.rtiles + rt) * (size_t)k * MT;
    const long long b0 = a.off0 + (long long)w * a.cols_per_wg;
    const long long b1 = min(b0 + (long long)a.cols_per_wg, a.B);
    for (long long o = b0 + threadIdx.x; o < b1; o += kThreads) {
        uint32_t acc[MT];
#pragma unroll
        for (int p = 0; p < MT; ++p) acc[p] = 0u;
        for (int j = 0; j < k; ++j) {
            const uint32_t x = src_ptr<MODE>(a, s, prog, j)[o];
            const ECG_CONST CoefTab* t = T + (size_t)j * MT;
            if constexpr (BIN) {
#pragma unroll
                for (int p = 0; p < MT; ++p) acc[p] ^= x & t[p].mask;
            } else {
                const Split sp = split(x);
#pragma unroll
                for (int p = 0; p < MT; ++p) acc[p] ^= gmul(t[p], sp);
            }
        }
#pragma unroll
        for (int p = 0; p < MT; ++p)
            if (p < nrows) dst_ptr<MODE>(a, s, prog, row0 + p)[o] = (uint8_t)(acc[p] & 0xffu);
    }
}

__global__ void __launch_bounds__(kThreads) fill_splitmix_kernel(uint8_t* dst, long long nbytes,
                                                                 unsigned long long seed,
                                                                 unsigned long long word_offset) {
    const long long nwords = nbytes >> 3;
    const long long stride = (long long)gridDim.x * kThreads;
    for (long long w = (long long)blockIdx.x * kThreads + threadIdx.x; w < ((nbytes + 7) >> 3); w += stride) {
        unsigned long long z = seed + (word_offset + (unsigned long long)w) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        if (w < nwords) {
            reinterpret_cast<unsigned long long*>(dst)[w] = z;
        } else {
            for (long long b = w * 8; b < nbytes; ++b) dst[b] = (uint8_t)(z >> (8 * (b - w * 8)));
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Dispatch

std::atomic<long long> g_opt[ECG_OPT_COUNT] = {};
std::atomic<int> g_opt_init{0};

void init_options() {
    if (g_opt_init.load(std::memory_order_acquire)) return;
    auto env = [](const char* n, long long d) {
        const char* e = getenv(n);
        return e ? atoll(e) : d;
    };
    g_opt[ECG_OPT_NT].store(env("ECG_NT", 3));
    g_opt[ECG_OPT_COLS_PER_WG].store(env("ECG_COLS_PER_WG", 0));
    g_opt[ECG_OPT_GRID_MAP].store(env("ECG_GRID_MAP", 3));
    // every staged call (r02 host_latency.py --sweep-zc: zero-copy with completion flags beats DMA staging
    // at every block size up to kStagedMaxBlock)
    g_opt[ECG_OPT_ZEROCOPY_BYTES].store(env("ECG_ZEROCOPY_BYTES", 8 << 20));
    g_opt[ECG_OPT_PROGRAM_CACHE].store(env("ECG_PROGRAM_CACHE", 4096));
    g_opt[ECG_OPT_MAP_GROUP].store(env("ECG_MAP_GROUP", 1));
    g_opt[ECG_OPT_LAT_DWORD_BYTES].store(env("ECG_LAT_DWORD_BYTES", 1 << 20));
    g_opt[ECG_OPT_CALL_WORKER].store(env("ECG_CALL_WORKER", 0));
    g_opt[ECG_OPT_ROW_SPLIT].store(env("ECG_ROW_SPLIT", 16));
    g_opt[ECG_OPT_GRAVEYARD].store(env("ECG_GRAVEYARD", 16384));
    g_opt[ECG_OPT_MT1_LDS_PAD].store(env("ECG_MT1_LDS_PAD", -1));
    g_opt_init.store(1, std::memory_order_release);
}

// Launchers return the status of THEIR launch (hipLaunchKernel's return value): the thread's sticky
// last error (hipGetLastError) also holds errors of earlier runtime calls the caller made and handled, and
// the library neither reads nor clears that state.
using Launcher = hipError_t (*)(const GfLaunch&, dim3, hipStream_t);

template <typename T>
struct NoDeduce {
    using type = T;
};

template <typename... P>
hipError_t launch_kernel_lds(void (*kernel)(P...), dim3 grid, dim3 block, unsigned lds, hipStream_t st,
                             typename NoDeduce<P>::type... args) {
    void* argv[] = {(void*)&args...};
    return hipLaunchKernel((const void*)kernel, grid, block, argv, lds, st);
}

template <typename... P>
hipError_t launch_kernel(void (*kernel)(P...), dim3 grid, dim3 block, hipStream_t st,
                         typename NoDeduce<P>::type... args) {
    return launch_kernel_lds(kernel, grid, block, 0, st, args...);
}

template <typename F>
hipError_t launch_with(F kernel, const GfLaunch& a, dim3 grid, hipStream_t st) {
    return launch_kernel(kernel, grid, dim3(kThreads), st, a);
}

// Single-output vector launches reserve dynamic LDS they never touch: the only effect is a cap on how many
// of their workgroups share a CU, and with it on how many block streams a CU keeps open at once.  The best
// cap falls as the input count grows (profiles/r05/occupancy/shapes_b4.log, shapes_k123.log: k -> 1 over
// 1 MiB blocks, one process, same buffers): 2-3 inputs +2-4 % at 12 KiB, 6 inputs +1-2 % at 20 KiB, 8-16
// inputs +2-6 % at 22-24 KiB; one step past each value the rate falls off a cliff (a 1 -> 1 copy already
// at 12 KiB: 0.80 -> 0.69, so it takes none).  Six-input pointer-table launches (config 3's scope flushes)
// do best one step higher than strided ones (+1.2-1.5 %, sweep_c3_box2.log, box3/sweep_c3.log).
// GENERAL launches of 3+ outputs (the encode) lose at every pad and take none; two-output launches: mt2_lds_pad;
// BINARY tiles of 8-9 outputs: gen_launch.
unsigned mt1_lds_pad(int k, bool ptrs) {
    const long long opt = g_opt[ECG_OPT_MT1_LDS_PAD].load(std::memory_order_relaxed);
    if (opt >= 0) return (unsigned)opt;
    if (k <= 1) return 0;
    if (k <= 3) return 12288;
    if (k == 4) return 16384;
    if (k == 5) return 0;
    if (k == 6) return ptrs ? 22528 : 20480;
    if (k == 7 || k == 9 || k == 10) return 22528;
    return 24576;
}

// Two-output launches (2-block repairs and 2-erasure decodes) take the same kind of cap once they read 8 or more
// inputs: pointer-table launches, both flavours, two processes each (profiles/r06/families/shape_probe/sp_pad2_*.log):
// 12 -> 2 0.722 -> 0.734-0.748 at 24 KiB, 20 -> 2 0.700-0.707 -> 0.725-0.727, 30 -> 2 0.702-0.710 -> 0.740-0.751,
// BINARY 12 / 16 -> 2 +2.5-3 %; 8-10 inputs +1-1.5 % at 20 KiB; 6 inputs none, and 28 KiB already falls off there.
// (Round 5 measured 0-2 % at 16-20 KiB on 10-input decodes and kept none.)  ECG_TUNE_PAD_MT2 builds take
// ECG_OPT_MT1_LDS_PAD for them too (tuning only).
unsigned mt2_lds_pad(int k) {
#ifdef ECG_TUNE_PAD_MT2
    const long long opt = g_opt[ECG_OPT_MT1_LDS_PAD].load(std::memory_order_relaxed);
    if (opt >= 0) return (unsigned)opt;
#endif
    return k <= 7 ? 0u : k <= 11 ? 20480u : 24576u;
}

template <int MT, int MODE, int NT, bool BIN>
hipError_t gen_launch(const GfLaunch& a, dim3 g, hipStream_t st) {
#ifdef ECG_TUNE_PAD_MT_LO  // tuning builds only: ECG_OPT_MT1_LDS_PAD caps launches of MT_LO..MT_HI outputs too
    if constexpr (MT >= ECG_TUNE_PAD_MT_LO && MT <= ECG_TUNE_PAD_MT_HI) {
        const long long opt = g_opt[ECG_OPT_MT1_LDS_PAD].load(std::memory_order_relaxed);
        return launch_kernel_lds(gf_vec_kernel<MT, MODE, NT, BIN>, g, dim3(kThreads), opt > 0 ? (unsigned)opt : 0u, st, a);
    }
#endif
    // BINARY tiles of 8-9 outputs (the composed PC / HPC / HVPC encodes, 16 -> 9 and 16 -> 8) run at 8 waves per
    // SIMD on 52-56 VGPRs and stream 24-25 blocks per workgroup; from 12 inputs a 20 KiB cap is +1.5-2.3 % (16 -> 9
    // in four of four runs, 16 -> 8, 12 -> 8; profiles/r06/families/shape_probe/sp_padw_*.log).  Wider BINARY tiles
    // (16 -> 16: 85 VGPRs, 5 waves) and GENERAL tiles of 3+ outputs lose under any cap.
    constexpr bool kWideBinCap = BIN && (MT == 8 || MT == 9);
    const unsigned lds = MT == 1 ? mt1_lds_pad(a.k, MODE == GF_MODE_PTRS)
                         : MT == 2 ? mt2_lds_pad(a.k)
                         : (kWideBinCap && a.k >= 12) ? 20480u : 0u;
    return launch_kernel_lds(gf_vec_kernel<MT, MODE, NT, BIN>, g, dim3(kThreads), lds, st, a);
}

template <int MODE, int NT, bool BIN>
Launcher gen_pick(int MT) {
    switch (MT) {
        case 1: return gen_launch<1, MODE, NT, BIN>;
        case 2: return gen_launch<2, MODE, NT, BIN>;
        case 3: return gen_launch<3, MODE, NT, BIN>;
        case 4: return gen_launch<4, MODE, NT, BIN>;
        case 5: return gen_launch<5, MODE, NT, BIN>;
        case 6: return gen_launch<6, MODE, NT, BIN>;
        case 7: return gen_launch<7, MODE, NT, BIN>;
        case 8: return gen_launch<8, MODE, NT, BIN>;
        default: break;
    }
    // wide BINARY tiles (kMaxMTBin): only the default NT policy is built (launch_gf runs them with it)
    if constexpr (BIN && NT == 3) {
        switch (MT) {
            case 9: return gen_launch<9, MODE, NT, BIN>;
            case 10: return gen_launch<10, MODE, NT, BIN>;
            case 11: return gen_launch<11, MODE, NT, BIN>;
            case 12: return gen_launch<12, MODE, NT, BIN>;
            case 13: return gen_launch<13, MODE, NT, BIN>;
            case 14: return gen_launch<14, MODE, NT, BIN>;
            case 15: return gen_launch<15, MODE, NT, BIN>;
            case 16: return gen_launch<16, MODE, NT, BIN>;
            default: break;
        }
    }
    return nullptr;
}

template <int MODE, int NT>
Launcher pick_vec_nt(const GfLaunch& a) {
    return a.binary ? gen_pick<MODE, NT, true>(a.MT) : gen_pick<MODE, NT, false>(a.MT);
}

template <int MODE>
Launcher pick_vec(const GfLaunch& a, int nt) {
    switch (nt & 3) {
        case 0: return pick_vec_nt<MODE, 0>(a);
        case 1: return pick_vec_nt<MODE, 1>(a);
        case 2: return pick_vec_nt<MODE, 2>(a);
        default: return pick_vec_nt<MODE, 3>(a);
    }
}

template <int MT, bool BIN, int KB>
hipError_t lat_dword_launch(const GfLaunch& a, dim3 g, hipStream_t st) {
    LatArgs<KB, MT> l;
    l.tabs = a.tabs;
    l.done_flags = a.done_flags;
    l.B = a.B;
    l.k = a.k;
    l.m = a.m;
    l.done_seq = a.done_seq;
    for (int u = 0; u < KB; ++u) l.src[u] = a.isrc[u < a.k ? u : 0];
    for (int p = 0; p < MT; ++p) l.dst[p] = a.idst[p < a.m ? p : 0];
    if (a.B <= kLatEagerBytes) return launch_kernel(gf_lat_dword_kernel<MT, BIN, KB, true>, g, dim3(kLatThreads), st, l);
    return launch_kernel(gf_lat_dword_kernel<MT, BIN, KB, false>, g, dim3(kLatThreads), st, l);
}

// input-count buckets of the latency kernel: exact for the BASELINE shapes (RS(6,4), RS(10,4) encode and
// decode, Azure-LRC(12,2,2) global rows), at most 3 padded inputs elsewhere
template <int MT, bool BIN>
Launcher pick_lat_k(int k) {
    if (k <= 4) return lat_dword_launch<MT, BIN, 4>;
    if (k <= 6) return lat_dword_launch<MT, BIN, 6>;
    if (k <= 8) return lat_dword_launch<MT, BIN, 8>;
    if (k <= 10) return lat_dword_launch<MT, BIN, 10>;
    if (k <= 12) return lat_dword_launch<MT, BIN, 12>;
    if (k <= 16) return lat_dword_launch<MT, BIN, 16>;
    return nullptr;
}

template <bool BIN>
Launcher pick_lat_dword_bin(int MT, int k) {
    switch (MT) {
        case 1: return pick_lat_k<1, BIN>(k);
        case 2: return pick_lat_k<2, BIN>(k);
        case 3: return pick_lat_k<3, BIN>(k);
        case 4: return pick_lat_k<4, BIN>(k);
        case 5: return pick_lat_k<5, BIN>(k);
        case 6: return pick_lat_k<6, BIN>(k);
        case 7: return pick_lat_k<7, BIN>(k);
        case 8: return pick_lat_k<8, BIN>(k);
        default: return nullptr;
    }
}

template <int MT, int MODE, bool BIN>
hipError_t byte_launch(const GfLaunch& a, dim3 g, hipStream_t st) {
    return launch_with(gf_byte_kernel<MT, MODE, BIN>, a, g, st);
}

template <int MODE, bool BIN>
Launcher pick_byte_bin(int MT) {
    switch (MT) {
        case 1: return byte_launch<1, MODE, BIN>;
        case 2: return byte_launch<2, MODE, BIN>;
        case 3: return byte_launch<3, MODE, BIN>;
        case 4: return byte_launch<4, MODE, BIN>;
        case 5: return byte_launch<5, MODE, BIN>;
        case 6: return byte_launch<6, MODE, BIN>;
        case 7: return byte_launch<7, MODE, BIN>;
        case 8: return byte_launch<8, MODE, BIN>;
        default: break;
    }
    if constexpr (BIN) {
        switch (MT) {
            case 9: return byte_launch<9, MODE, BIN>;
            case 10: return byte_launch<10, MODE, BIN>;
            case 11: return byte_launch<11, MODE, BIN>;
            case 12: return byte_launch<12, MODE, BIN>;
            case 13: return byte_launch<13, MODE, BIN>;
            case 14: return byte_launch<14, MODE, BIN>;
            case 15: return byte_launch<15, MODE, BIN>;
            case 16: return byte_launch<16, MODE, BIN>;
            default: break;
        }
    }
    return nullptr;
}

template <int MODE>
Launcher pick_byte(const GfLaunch& a) {
    return a.binary ? pick_byte_bin<MODE, true>(a.MT) : pick_byte_bin<MODE, false>(a.MT);
}

}  // namespace

long long get_option(int opt) {
    init_options();
    if (opt < 0 || opt >= ECG_OPT_COUNT) return -1;
    return g_opt[opt].load();
}

int set_option(int opt, long long value) {
    init_options();
    if (opt < 0 || opt >= ECG_OPT_COUNT) return -1;
    if (opt == ECG_OPT_NT && (value < 0 || value > 3)) return -1;
    if (opt == ECG_OPT_COLS_PER_WG && (value < 0 || (value % kThreads) != 0)) return -1;
    if (opt == ECG_OPT_GRID_MAP && (value < 0 || value > 3)) return -1;
    if (opt == ECG_OPT_ZEROCOPY_BYTES && value < 0) return -1;
    if (opt == ECG_OPT_PROGRAM_CACHE && value < 2) return -1;
    if (opt == ECG_OPT_MAP_GROUP && (value < 1 || value > (1 << 20))) return -1;
    if (opt == ECG_OPT_LAT_DWORD_BYTES && value < 0) return -1;
    if (opt == ECG_OPT_CALL_WORKER && (value < 0 || value > 1000000)) return -1;  // idle limit <= 1 s
    if (opt == ECG_OPT_ROW_SPLIT && value < 0) return -1;
    if (opt == ECG_OPT_GRAVEYARD && value < 1) return -1;
    if (opt == ECG_OPT_MT1_LDS_PAD && (value < -1 || value > 65536)) return -1;
    g_opt[opt].store(value);
    return 0;
}

// Grid-map auto rule (profiles/r01/shape_sweep.py, every k_in x m_out shape): when the outputs are blocks
// of the input stripes themselves (encode: [S][k+m][B]), XCD-contiguous chunks (map 1) are 1-3 % faster;
// when they go to a separate buffer (decode / repair / merge outputs), putting stripe s on XCD s % 8
// (map 2) is 2-6 % faster.  Pointer-table launches have no single layout: the engine, which builds the
// table, passes grid_map = 2 when every call's outputs lie apart from its inputs (a batch scope's repairs
// and merges: 2-3 % faster in one process on the same buffers, profiles/r05/ptrs_map/), else they take map 1.
static bool outputs_in_stripe(const GfLaunch& a, int mode) {
    if (mode == GF_MODE_PTRS) return a.grid_map != 2;
    if (mode != GF_MODE_STRIDED) return true;
    const uint8_t* o = a.out_base;
    return a.out_sstride == a.in_sstride && o >= a.in_base && o < a.in_base + a.in_sstride;
}

// Process-wide traffic counters (ecg_traffic_counters): region-product kernels launched, and the bytes they move
// as planned -- every row tile reads the launch's k inputs, every output is written once: S * B * (rtiles * k + m)
// per region product.  Relaxed atomics: two uncontended adds per launch.
std::atomic<long long> g_launched{0}, g_moved{0};

void launch_traffic(long long* launches, long long* bytes) {
    if (launches) *launches = g_launched.load(std::memory_order_relaxed);
    if (bytes) *bytes = g_moved.load(std::memory_order_relaxed);
}

hipError_t launch_gf(const GfLaunch& base, int mode, bool vec_ok, hipStream_t st, int* n_wg) {
    if (n_wg) *n_wg = 0;
    if (base.k < 1 || base.m < 1 || base.S < 1 || base.B < 0 || base.MT < 1 ||
        base.MT > (base.binary ? kMaxMTBin : kMaxMT))
        return hipErrorInvalidValue;
    if ((mode == GF_MODE_INLINE || mode == GF_MODE_INLINE_LAT) &&
        (base.S != 1 || base.k > kInlineSrc || base.m > kInlineDst))
        return hipErrorInvalidValue;
    if (base.B == 0) return hipSuccess;
    init_options();
    GfLaunch a = base;
    const long long vec_bytes = vec_ok ? (a.B & ~15LL) : 0;
    g_launched.fetch_add((vec_bytes > 0) + (vec_bytes < a.B), std::memory_order_relaxed);
    g_moved.fetch_add((long long)a.S * a.B * ((long long)a.rtiles * a.k + a.m), std::memory_order_relaxed);
    if (mode == GF_MODE_INLINE_LAT && vec_bytes == a.B && a.B <= g_opt[ECG_OPT_LAT_DWORD_BYTES].load() &&
        a.k <= kLatMaxSrc && a.rtiles == 1 && a.MT <= kMaxMT) {
        // small zero-copy call: 4 bytes per lane (gf_lat_dword_kernel)
        const long long gx = ((a.B >> 2) + kLatThreads - 1) / kLatThreads;
        Launcher l = a.binary ? pick_lat_dword_bin<true>(a.MT, a.k) : pick_lat_dword_bin<false>(a.MT, a.k);
        if (!l) return hipErrorInvalidValue;
        const hipError_t e = l(a, dim3((unsigned)gx), st);
        if (e != hipSuccess) return e;
        if (n_wg) *n_wg = (int)gx;
        return hipSuccess;
    }
    if (vec_bytes > 0) {
        const long long ncols = vec_bytes >> 4;
        long long cpw = g_opt[ECG_OPT_COLS_PER_WG].load();
        if (cpw <= 0) cpw = kThreads;  // 2 KiB of every block per workgroup (measured best, r01 microbench)
        if (ncols < cpw) cpw = ((ncols + kThreads - 1) / kThreads) * kThreads;
        a.cols_per_wg = (int)cpw;
        a.wg_per_stripe = (int)((ncols + cpw - 1) / cpw);
        a.off0 = 0;
        const long long gx = (long long)a.S * a.wg_per_stripe;
        if (gx > 0x7fffffffLL) return hipErrorInvalidConfiguration;
        long long gm = g_opt[ECG_OPT_GRID_MAP].load();
        if (gm == 3) gm = outputs_in_stripe(a, mode) ? 1 : 2;
        long long G = g_opt[ECG_OPT_MAP_GROUP].load();
        while (G > 1 && a.S % (8 * G) != 0) G >>= 1;  // the largest power-of-two divisor run that tiles S
        if (gm == 2 && a.S % (8 * G) != 0) gm = 1;
        a.grid_map = (gm == 1 && gx % 8 == 0) ? 1 : (gm == 2) ? 2 : 0;
        a.map_group = (int)G;
        const int nt = a.MT > kMaxMT ? 3 : (int)g_opt[ECG_OPT_NT].load();  // wide tiles: built for the default only
        Launcher l = nullptr;
        switch (mode) {
            case GF_MODE_INLINE: l = pick_vec<GF_MODE_INLINE>(a, nt); break;
            case GF_MODE_INLINE_LAT: l = pick_vec<GF_MODE_INLINE_LAT>(a, nt); break;
            case GF_MODE_PTRS: l = pick_vec<GF_MODE_PTRS>(a, nt); break;
            case GF_MODE_STRIDED: l = pick_vec<GF_MODE_STRIDED>(a, nt); break;
            default: return hipErrorInvalidValue;
        }
        if (!l) return hipErrorInvalidValue;
        if (a.done_flags && (mode != GF_MODE_INLINE_LAT || vec_bytes < a.B)) return hipErrorInvalidValue;
        const hipError_t e = l(a, dim3((unsigned)gx, (unsigned)a.rtiles), st);
        if (e != hipSuccess) return e;
        if (n_wg) *n_wg = (int)(gx * a.rtiles);
    }
    if (a.done_flags && vec_bytes < a.B) return hipErrorInvalidValue;  // the byte kernel posts no flags
    if (vec_bytes < a.B) {
        const long long nbytes = a.B - vec_bytes;
        long long bpw = 16LL * kThreads;
        if (nbytes < bpw) bpw = ((nbytes + kThreads - 1) / kThreads) * kThreads;
        a.cols_per_wg = (int)bpw;
        a.wg_per_stripe = (int)((nbytes + bpw - 1) / bpw);
        a.off0 = vec_bytes;
        a.grid_map = 0;
        const long long gx = (long long)a.S * a.wg_per_stripe;
        if (gx > 0x7fffffffLL) return hipErrorInvalidConfiguration;
        Launcher l = nullptr;
        switch (mode) {
            case GF_MODE_INLINE:
            case GF_MODE_INLINE_LAT: l = pick_byte<GF_MODE_INLINE>(a); break;
            case GF_MODE_PTRS: l = pick_byte<GF_MODE_PTRS>(a); break;
            case GF_MODE_STRIDED: l = pick_byte<GF_MODE_STRIDED>(a); break;
            default: return hipErrorInvalidValue;
        }
        if (!l) return hipErrorInvalidValue;
        const hipError_t e = l(a, dim3((unsigned)gx, (unsigned)a.rtiles), st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_call_worker(const WorkerArgs& a, int workgroups, hipStream_t st) {
    if (workgroups < 1 || workgroups > kWorkerMaxWG) return hipErrorInvalidValue;
    return launch_kernel(gf_call_worker_kernel, dim3((unsigned)workgroups), dim3(kLatThreads), st, a);
}

hipError_t launch_fill_splitmix(void* dst, long long nbytes, unsigned long long seed,
                                unsigned long long word_offset, hipStream_t st) {
    if (nbytes <= 0) return hipSuccess;
    const long long nwords = (nbytes + 7) >> 3;
    long long blocks = (nwords + kThreads - 1) / kThreads;
    if (blocks > 8192) blocks = 8192;
    return launch_kernel(fill_splitmix_kernel, dim3((unsigned)blocks), dim3(kThreads), st, (uint8_t*)dst, nbytes,
                         seed, word_offset);
}

void make_coef_tab(int c, CoefTab* t) {
    c &= 0xff;
    uint8_t e0[8], e1[8], e2[4];
    for (int e = 0; e < 8; ++e) {
        e0[e] = (uint8_t)gf::mul(c, e);
        e1[e] = (uint8_t)gf::mul(c, e << 3);
    }
    for (int e = 0; e < 4; ++e) e2[e] = (uint8_t)gf::mul(c, e << 6);
    auto pack = [](const uint8_t* b) {
        return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    };
    t->t0lo = pack(e0);
    t->t0hi = pack(e0 + 4);
    t->t1lo = pack(e1);
    t->t1hi = pack(e1 + 4);
    t->t2 = pack(e2);
    t->mask = (c == 1) ? 0xffffffffu : 0u;
    t->pad0 = 0u;
    t->pad1 = 0u;
}

}  // namespace ecg
