// GF(2^8) region-product kernels for MI355X (gfx950, CDNA4).
//
// out_p[x] = XOR_j c[p][j] * in_j[x] over GF(2^8)/0x11d, for p < m, j < k, every byte x of a block.
//
// Data path (HBM-bound, no MFMA -- byte-field XOR-multiply, not a dense contraction):
//   * each lane owns one 16-byte column of every block: one global_load_dwordx4 per input block,
//     64 lanes = 1 KiB contiguous per wave-instruction, 4 inputs in flight per unrolled step;
//   * m_out accumulators of 16 bytes stay in VGPRs, so every input byte is read from HBM once and
//     every output byte written once ((k + m) * B bytes per stripe: the algorithmic minimum);
//   * the multiply is three v_perm_b32 table lookups per dword (bit fields [2:0], [5:3], [7:6]) with
//     the per-coefficient tables in SGPRs (scalar loads of a 32-byte CoefTab), folded with gfx950's
//     v_bitop3_b32 (3-input XOR); the bit-field split of an input dword is shared by all m outputs;
//   * straight-line code (no per-coefficient branches); matrices whose entries are all 0/1
//     (perform_addition, LRC local rows, PC merges) take a BINARY flavour: one v_bitop3
//     acc ^ (x & mask) per coefficient-dword.
// VALU cost per 16-byte column: 20 ops to split one input, ~18 per coefficient (GENERAL) or 4
// (BINARY); for RS(10,4) encode ~1000 ops per 160 data bytes, ~35 % of gfx950's integer issue rate
// at the HBM roofline.
#include "gf_kernels.hpp"
#include "gf256.hpp"

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
    if constexpr (MODE == GF_MODE_INLINE) {
        return a.isrc[j];
    } else if constexpr (MODE == GF_MODE_PTRS) {
        return cst(a.src_ptrs)[(size_t)s * a.k + j];
    } else {
        return a.in_base + (long long)s * a.in_sstride + (long long)cst(a.src_ids)[prog * a.k + j] * a.in_bstride;
    }
}

template <int MODE>
__device__ __forceinline__ uint8_t* dst_ptr(const GfLaunch& a, int s, int prog, int p) {
    if constexpr (MODE == GF_MODE_INLINE) {
        return a.idst[p];
    } else if constexpr (MODE == GF_MODE_PTRS) {
        return cst(a.dst_ptrs)[(size_t)s * a.m + p];
    } else {
        return a.out_base + (long long)s * a.out_sstride + (long long)cst(a.dst_ids)[prog * a.m + p] * a.out_bstride;
    }
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// gfx950 v_bitop3_b32 with truth table 0x96 = a ^ b ^ c in one VALU op.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void load16(const uint8_t* p, uint32_t (&x)[4]) {
    u32x4 v;
    if constexpr (NT) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else v = *reinterpret_cast<const u32x4*>(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
}

template <bool NT>
__device__ __forceinline__ void store16(uint8_t* p, const uint32_t (&x)[4]) {
    u32x4 v;
    v.x = x[0]; v.y = x[1]; v.z = x[2]; v.w = x[3];
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
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

// GENERAL flavour: U inputs (U = 1, 2 or 4) folded into MT accumulators.  Straight-line: every
// coefficient goes through the tables (c = 0 and c = 1 tables are exact), products of input pairs
// are folded with one v_bitop3 each so a coefficient costs 3 perm + 1.5 bitop3 per dword.
template <int MT, int U>
__device__ __forceinline__ void fold_general(const uint32_t (&x)[U][4], const ECG_CONST CoefTab* t,
                                             uint32_t (&acc)[MT][4]) {
    if constexpr (U == 1) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const Split s0 = split(x[0][d]);
#pragma unroll
            for (int p = 0; p < MT; ++p) acc[p][d] ^= gmul(t[p], s0);
        }
    } else {
#pragma unroll
        for (int u = 0; u < U; u += 2) {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const Split s0 = split(x[u][d]);
                const Split s1 = split(x[u + 1][d]);
#pragma unroll
                for (int p = 0; p < MT; ++p)
                    acc[p][d] = xor3(acc[p][d], gmul(t[u * MT + p], s0), gmul(t[(u + 1) * MT + p], s1));
            }
        }
    }
}

// BINARY flavour (every coefficient 0 or 1: perform_addition, LRC local rows, PC merges):
// acc ^= x & mask in one v_bitop3 (LUT index = S0<<2 | S1<<1 | S2, so a ^ (b & c) = 0x78), mask = 0 or ~0 from SGPRs.
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

// Vector path: bytes [0, 16 * floor(B / 16)) of every block; all pointers 16-byte aligned.
// grid.x = S * wg_per_stripe (stripe-major), grid.y = row tiles of MT outputs.
template <int MT, int MODE, bool NT, bool BIN>
__global__ void __launch_bounds__(kThreads, (MT <= 4 ? 6 : 4)) gf_vec_kernel(const GfLaunch a) {
    const int s = blockIdx.x / a.wg_per_stripe;
    const int w = blockIdx.x - s * a.wg_per_stripe;
    const int rt = blockIdx.y;
    const int prog = a.prog_of_stripe ? cst(a.prog_of_stripe)[s] : 0;
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
        for (; j + 4 <= k; j += 4) {
            uint32_t x[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off, x[u]);
            fold<MT, 4, BIN>(x, T + (size_t)j * MT, acc);
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
}

// Byte path: bytes [off0, B) (tails, unaligned pointers).  cols_per_wg = bytes per workgroup.
template <int MT, int MODE, bool BIN>
__global__ void __launch_bounds__(kThreads) gf_byte_kernel(const GfLaunch a) {
    const int s = blockIdx.x / a.wg_per_stripe;
    const int w = blockIdx.x - s * a.wg_per_stripe;
    const int rt = blockIdx.y;
    const int prog = a.prog_of_stripe ? cst(a.prog_of_stripe)[s] : 0;
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

template <int MT, int MODE, bool BIN>
hipError_t dispatch_vec(const GfLaunch& a, dim3 grid, bool nt, hipStream_t st) {
    if (nt) hipLaunchKernelGGL((gf_vec_kernel<MT, MODE, true, BIN>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((gf_vec_kernel<MT, MODE, false, BIN>), grid, dim3(kThreads), 0, st, a);
    return hipGetLastError();
}

template <int MODE, bool BIN>
hipError_t dispatch_vec_mt(const GfLaunch& a, dim3 grid, bool nt, hipStream_t st) {
    switch (a.MT) {
        case 1: return dispatch_vec<1, MODE, BIN>(a, grid, nt, st);
        case 2: return dispatch_vec<2, MODE, BIN>(a, grid, nt, st);
        case 3: return dispatch_vec<3, MODE, BIN>(a, grid, nt, st);
        case 4: return dispatch_vec<4, MODE, BIN>(a, grid, nt, st);
        case 5: return dispatch_vec<5, MODE, BIN>(a, grid, nt, st);
        case 6: return dispatch_vec<6, MODE, BIN>(a, grid, nt, st);
        case 7: return dispatch_vec<7, MODE, BIN>(a, grid, nt, st);
        case 8: return dispatch_vec<8, MODE, BIN>(a, grid, nt, st);
        default: return hipErrorInvalidValue;
    }
}

template <int MODE>
hipError_t dispatch_vec_bin(const GfLaunch& a, dim3 grid, bool nt, hipStream_t st) {
    return a.binary ? dispatch_vec_mt<MODE, true>(a, grid, nt, st) : dispatch_vec_mt<MODE, false>(a, grid, nt, st);
}

template <int MODE, bool BIN>
hipError_t dispatch_byte_mt(const GfLaunch& a, dim3 grid, hipStream_t st) {
#define ECG_BYTE_CASE(N) \
    case N: hipLaunchKernelGGL((gf_byte_kernel<N, MODE, BIN>), grid, dim3(kThreads), 0, st, a); break;
    switch (a.MT) {
        ECG_BYTE_CASE(1) ECG_BYTE_CASE(2) ECG_BYTE_CASE(3) ECG_BYTE_CASE(4)
        ECG_BYTE_CASE(5) ECG_BYTE_CASE(6) ECG_BYTE_CASE(7) ECG_BYTE_CASE(8)
        default: return hipErrorInvalidValue;
    }
#undef ECG_BYTE_CASE
    return hipGetLastError();
}

template <int MODE>
hipError_t dispatch_byte_bin(const GfLaunch& a, dim3 grid, hipStream_t st) {
    return a.binary ? dispatch_byte_mt<MODE, true>(a, grid, st) : dispatch_byte_mt<MODE, false>(a, grid, st);
}

bool use_nt_default() {
    static const int v = [] {
        const char* e = getenv("ECG_NT");
        return e ? atoi(e) : 1;
    }();
    return v != 0;
}

}  // namespace

hipError_t launch_gf(const GfLaunch& base, int mode, bool vec_ok, hipStream_t st) {
    if (base.k < 1 || base.m < 1 || base.S < 1 || base.B < 0 || base.MT < 1 || base.MT > kMaxMT)
        return hipErrorInvalidValue;
    if (mode == GF_MODE_INLINE && (base.S != 1 || base.k > kInlineSrc || base.m > kInlineDst))
        return hipErrorInvalidValue;
    if (base.B == 0) return hipSuccess;
    GfLaunch a = base;
    const long long vec_bytes = vec_ok ? (a.B & ~15LL) : 0;
    if (vec_bytes > 0) {
        const long long ncols = vec_bytes >> 4;
        long long cpw = 4LL * kThreads;                       // 16 KiB of every block per workgroup
        if (ncols < cpw) cpw = ((ncols + kThreads - 1) / kThreads) * kThreads;
        a.cols_per_wg = (int)cpw;
        a.wg_per_stripe = (int)((ncols + cpw - 1) / cpw);
        a.off0 = 0;
        const long long gx = (long long)a.S * a.wg_per_stripe;
        if (gx > 0x7fffffffLL) return hipErrorInvalidConfiguration;
        dim3 grid((unsigned)gx, (unsigned)a.rtiles);
        const bool nt = use_nt_default();
        hipError_t e;
        switch (mode) {
            case GF_MODE_INLINE: e = dispatch_vec_bin<GF_MODE_INLINE>(a, grid, nt, st); break;
            case GF_MODE_PTRS: e = dispatch_vec_bin<GF_MODE_PTRS>(a, grid, nt, st); break;
            case GF_MODE_STRIDED: e = dispatch_vec_bin<GF_MODE_STRIDED>(a, grid, nt, st); break;
            default: return hipErrorInvalidValue;
        }
        if (e != hipSuccess) return e;
    }
    if (vec_bytes < a.B) {
        const long long nbytes = a.B - vec_bytes;
        long long bpw = 16LL * kThreads;
        if (nbytes < bpw) bpw = ((nbytes + kThreads - 1) / kThreads) * kThreads;
        a.cols_per_wg = (int)bpw;
        a.wg_per_stripe = (int)((nbytes + bpw - 1) / bpw);
        a.off0 = vec_bytes;
        const long long gx = (long long)a.S * a.wg_per_stripe;
        if (gx > 0x7fffffffLL) return hipErrorInvalidConfiguration;
        dim3 grid((unsigned)gx, (unsigned)a.rtiles);
        hipError_t e;
        switch (mode) {
            case GF_MODE_INLINE: e = dispatch_byte_bin<GF_MODE_INLINE>(a, grid, st); break;
            case GF_MODE_PTRS: e = dispatch_byte_bin<GF_MODE_PTRS>(a, grid, st); break;
            case GF_MODE_STRIDED: e = dispatch_byte_bin<GF_MODE_STRIDED>(a, grid, st); break;
            default: return hipErrorInvalidValue;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_fill_splitmix(void* dst, long long nbytes, unsigned long long seed,
                                unsigned long long word_offset, hipStream_t st) {
    if (nbytes <= 0) return hipSuccess;
    const long long nwords = (nbytes + 7) >> 3;
    long long blocks = (nwords + kThreads - 1) / kThreads;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, st,
                       (uint8_t*)dst, nbytes, seed, word_offset);
    return hipGetLastError();
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
