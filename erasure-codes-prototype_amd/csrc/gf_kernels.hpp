// Device-side GF(2^8) region-product kernels for gfx950 (CDNA4) and their launch descriptors.
//
// One primitive covers every byte operation on the reference's hot path:
//   out_p = XOR_j  c[p][j] * in_j        (bytewise, GF(2^8) / 0x11d)
// jerasure_matrix_encode (a1), the dot products of jerasure_matrix_decode (a3, composed on the host
// into one matrix), perform_addition (a8, all-ones rows), partial encode / partial decode (a9/a10,
// sub-matrices) and galois_region_xor (a7, a 1x2 all-ones product) are all instances.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ecg.h"

namespace ecg {

// Per-coefficient multiply tables for v_perm_b32 (one 32-byte record, loaded into SGPRs).
// A byte b is split into bit fields b[2:0], b[5:3], b[7:6]; c*b = T0[b&7] ^ T1[(b>>3)&7] ^ T2[b>>6]
// (GF multiplication by a constant is linear over GF(2)).  T0/T1 have 8 one-byte entries (two dwords
// each, the v_perm 8-byte pool), T2 has 4 (one dword).
struct alignas(32) CoefTab {
    uint32_t t0lo, t0hi;  // c * e        for e = 0..7
    uint32_t t1lo, t1hi;  // c * (e << 3)
    uint32_t t2;          // c * (e << 6) for e = 0..3
    uint32_t mask;        // BINARY flavour: 0xffffffff if c == 1, 0 if c == 0
    uint32_t pad0, pad1;
};

enum GfMode : int {
    GF_MODE_INLINE = 0,   // S == 1, pointers carried in the kernel arguments
    GF_MODE_PTRS = 1,     // device pointer tables src_ptrs[S][k], dst_ptrs[S][m]
    GF_MODE_STRIDED = 2,  // base + stripe/block strides + per-program block ids
    GF_MODE_INLINE_LAT = 3,  // INLINE for latency-bound calls on host memory read over PCIe (zero-copy
                             // host tier): a lane issues all of its k <= 16 input loads before the first
                             // use -- one PCIe round trip instead of one per group of loads
};

constexpr int kInlineSrc = 128;
constexpr int kInlineDst = 32;
constexpr int kMaxMT = 8;       // output rows per row tile (GENERAL flavour)
constexpr int kMaxMTBin = 16;   // BINARY flavour (one v_bitop3 per coefficient-dword): a composed product-code
                                // call's 9-16 XOR rows read every input once (codes.cpp finish_plan)
#ifndef ECG_TPB
#define ECG_TPB 128
#endif
constexpr int kLatThreads = 256;  // dword columns per workgroup of the small-call latency kernel
constexpr int kLatMaxSrc = 16;    // inputs it loads up front
constexpr long long kLatEagerBytes = 16 << 10;  // blocks up to this size take its EAGER form
constexpr int kThreads = ECG_TPB;  // threads per workgroup (2 waves of 64, r01 tuning); ECG_TPB only for tuning builds

struct GfLaunch {
    // programs: [nprog][rtiles][k][MT] tables, [nprog][k] src ids, [nprog][m] dst ids
    const CoefTab* tabs;
    const int* src_ids;
    const int* dst_ids;
    const int* prog_of_stripe;   // [S] or nullptr (program 0 for every stripe)
    const int* stripe_of;        // [S] or nullptr: launch stripe i addresses stripe stripe_of[i] (STRIDED)
    int row_split;               // STRIDED: 0, or R -> launch stripe i is row i % R of stripe i / R (program
                                 // prog_of_stripe[i / R] * R + i % R); S counts launch stripes
    // GF_MODE_STRIDED
    const uint8_t* in_base;
    uint8_t* out_base;
    long long in_sstride, in_bstride, out_sstride, out_bstride;
    // GF_MODE_PTRS
    const uint8_t* const* src_ptrs;
    uint8_t* const* dst_ptrs;
    // GF_MODE_INLINE
    const uint8_t* isrc[kInlineSrc];
    uint8_t* idst[kInlineDst];
    long long B;         // block size in bytes
    long long off0;      // byte offset this launch starts at (tail launches)
    int k, m, S;
    int MT, rtiles;
    int binary;          // every coefficient is 0 or 1 -> BINARY kernel flavour
    int grid_map;        // 0 linear, 1 XCD-contiguous workgroup -> chunk mapping, 2 stripe groups per XCD.
                         // launch_gf sets it; on entry, for GF_MODE_PTRS only, 2 tells the auto rule that
                         // every call's outputs lie apart from its inputs (engine.cpp outputs_apart)
    int map_group;       // grid_map 2: G adjacent stripes per XCD group (S % (8 G) == 0)
    int wg_per_stripe;
    int cols_per_wg;     // 16-byte columns per workgroup (vector path) / bytes per workgroup (byte path)
    // GF_MODE_INLINE_LAT only: completion flags in mapped host memory.  When set, every workgroup writes
    // done_seq into done_flags[blockIdx.y * gridDim.x + blockIdx.x] after its stores are visible to the
    // host (system-scope release), so a synchronous host call can poll them instead of synchronizing
    // the stream.  Needs the vector path to cover every byte (no tail launch).
    unsigned* done_flags;
    unsigned done_seq;
};

// ---- resident call worker (ECG_OPT_CALL_WORKER) ----
// Small synchronous host-tier calls can skip the launch: a resident kernel on its own high-priority
// stream polls a ring of descriptors in pinned host memory and runs each call as the latency kernel
// would.  A descriptor is four 64-byte lines; dword 0 of every line is the call's sequence number and the
// host writes it last, so the worker takes a descriptor only when all four lines carry the number it
// waits for.  The other 60 dwords hold the payload in order (worker_pos maps payload index -> dword).
constexpr int kWorkerSlots = 4;     // ring slots (one call in flight: the engine serialises the worker)
constexpr int kWorkerMaxWG = 16;    // workgroups of a worker: blocks up to 16 KiB in one pass of 4-byte lanes
constexpr int kWorkerMaxSrc = 16;   // inputs per call
constexpr int kWorkerMaxRows = 4;   // outputs per call (one row tile)
struct alignas(256) WorkerDesc {
    unsigned w[64];
};
enum WorkerField : int {  // payload indices
    WF_K = 0, WF_M = 1, WF_B = 2, WF_BINARY = 3, WF_TABS = 4,  // tabs: 2 dwords
    WF_IN = 8,                                                // 16 input pointers, 2 dwords each
    WF_OUT = WF_IN + 2 * kWorkerMaxSrc,                       // 4 output pointers
    WF_END = WF_OUT + 2 * kWorkerMaxRows
};
static_assert(WF_END <= 60, "worker payload fits 60 dwords");
__host__ __device__ constexpr int worker_pos(int q) { return q + 1 + q / 15; }

struct WorkerArgs {
    const WorkerDesc* ring;  // [kWorkerSlots], pinned host (device view)
    unsigned* flags;         // [kWorkerSlots][kWorkerMaxWG], pinned host: flag of (call, workgroup) = seq
    const unsigned* stop;    // pinned host: nonzero = exit at the next poll
    WorkerDesc* mbox;        // [kWorkerSlots] device: the leader's copy of a descriptor for the others
    unsigned* mbseq;         // [kWorkerSlots + 1] device: sequence number per mailbox slot, then the exit word
    unsigned* exit_info;     // [kWorkerMaxWG] pinned host: `gen` once the workgroup has exited
    unsigned start_seq, gen, max_polls;
    unsigned long long idle_ticks, life_ticks;  // wall-clock ticks (hipDeviceAttributeWallClockRate, kHz)
};
hipError_t launch_call_worker(const WorkerArgs& a, int workgroups, hipStream_t stream);

// Runtime tuning options (ecg_set_option): see ECG_OPT_* in include/ecg.h.
long long get_option(int opt);
int set_option(int opt, long long value);

// Launch the region product over bytes [0, B) of every stripe.  `vec_ok` = every block pointer is
// 16-byte aligned (the host checks); otherwise the byte path covers everything.  Returns a hipError_t.
hipError_t launch_gf(const GfLaunch& base, int mode, bool vec_ok, hipStream_t stream, int* n_wg = nullptr);
// Region-product kernels launch_gf has launched in this process, and the bytes they move as planned.
void launch_traffic(long long* launches, long long* bytes);

// Deterministic synthetic bytes: 8-byte word w = splitmix64(seed + (word_offset + w) * golden).
hipError_t launch_fill_splitmix(void* dst, long long nbytes, unsigned long long seed,
                                unsigned long long word_offset, hipStream_t stream);

// Host-side table construction for coefficient c (product GF arithmetic, gf256.hpp).
void make_coef_tab(int c, CoefTab* out);

}  // namespace ecg
