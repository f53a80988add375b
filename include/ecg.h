/*
 * ecg.h — C ABI of the MI355X (gfx950) erasure-coding engine (libecg.so).
 *
 * Drop-in boundary for hhlgt/erasure-codes-prototype's hot path.  Three tiers:
 *
 *  1. Jerasure-compatible tier — the exact C API the reference links (project/CmakeLists.txt:116-134,
 *     "Jerasure gf_complete"), same arguments and semantics, w = 8 only.  Region arguments are HOST
 *     pointers (char** of B-byte buffers, as the proxy passes them: proxy.cpp:335-346); the bytes are
 *     staged through HBM and computed by the HIP kernels.  The reference's src/ec/{rs,lrc,pc,erasure_code}.cpp can be
 *     relinked against these symbols unchanged through the shim headers in include/jerasure_shim/.
 *  2. Device / batched tier — the same operations over HBM-resident blocks, asynchronous on a HIP
 *     stream, and batches of S stripes in one launch (what bench.py drives).
 *  3. ErasureCode facade — handles mirroring the reference's ErasureCode class hierarchy
 *     (project/include/ec/erasure_code.h:60-129) as built by ec_factory (project/src/metadata.cpp:48-77):
 *     RS, EnlargedRS, the five LRCs and the three product codes, with encode / decode /
 *     encode_partial_blocks_for_{encoding,decoding} / perform_addition.
 *
 * Status codes: where the reference function returns void, the ABI returns int (0 = done).  The
 * reference prints and returns on bad input ("[Decode] Undecodable!" rs.cpp:30-33, "invalid! %d mod %d"
 * erasure_code.cpp:73-76); the ABI returns the matching negative code instead and never exits.
 * Thread-safety: every entry point may be called concurrently from different threads (the proxy runs
 * EC calls on detached threads, proxy.cpp:416-419); the only shared state is a mutex-protected
 * coefficient-table cache.
 */
#ifndef ECG_H
#define ECG_H

#include <stddef.h> /* size_t (ecg_batch_scratch) */

#ifdef __cplusplus
extern "C" {
#endif

#define ECG_OK 0
#define ECG_EUNDECODABLE (-1) /* jerasure_matrix_decode returns -1; reference prints "[Decode] Failed!" */
#define ECG_EINVAL (-2)       /* bad arguments (w != 8, k/m out of range, block_num % parity_num != 0) */
#define ECG_EHIP (-3)         /* HIP runtime error; see ecg_last_error() */
#define ECG_EUNPINNED (-4)    /* Cauchy m == 2 needs Jerasure's cbest_8 table, not available offline */
#define ECG_ENOMEM (-5)

const char* ecg_last_error(void);  /* thread-local message for the last ECG_EHIP */
int ecg_version(void);             /* 100 * major + minor */
int ecg_device_count(void);
int ecg_set_device(int device);    /* selects the HIP device for the calling thread */
void ecg_free(void* p);            /* frees matrices returned by this library (malloc'd, like Jerasure) */
int ecg_program_cache_size(void);  /* programs cached for the current device (diagnostics) */
/* Evicted program tables of the current device not yet freed (diagnostics).  An evicted set is freed once
 * its launches have completed, proven by an event the library records on each stream the set ran on the
 * next time a caller hands it that stream (the library never names a caller stream after the call that
 * passed it returns: callers may destroy their streams at any time).  Sets whose streams are not seen again
 * wait in a bounded graveyard, emptied by one device synchronize when it grows past ECG_OPT_GRAVEYARD sets
 * (default 16384), or by ecg_program_sets_reclaim. */
int ecg_program_sets_retiring(void);
/* Synchronize the current device and free every evicted program set no call still holds (e.g. at idle, or
 * after a burst of per-request streams).  Returns the sets still retiring after it. */
int ecg_program_sets_reclaim(void);
/* Host-tier contexts (stream + device scratch + pinned staging) created so far for the current device
 * (diagnostics).  Contexts are pooled and leased per call, so this is bounded by the most host-tier calls
 * ever in flight at once, not by the number of threads that called (the reference's proxy starts a
 * thread per request, proxy.cpp:416-419). */
int ecg_host_contexts(void);
/* Resident call worker of the current device (ECG_OPT_CALL_WORKER), diagnostics: calls it completed,
 * kernel launches (generations started), generations relaunched under a waiting call, and whether it is
 * off right now (1) or not (0): off for good if it could not be set up, or for a cooldown (1 s, doubling per
 * consecutive timeout up to 64 s) after a call did not complete within 100 ms; calls then take the launch
 * path.  Any pointer may be NULL. */
int ecg_call_worker_stats(long long* calls, long long* launches, long long* relaunches, int* disabled);
/* The HIP runtime's pinned-transfer threshold for pageable host memory, in bytes, as this process runs
 * it: GPU_PINNED_MIN_XFER_SIZE (MiB) from the environment, default 1 MiB.  A pageable hipMemcpy of more
 * than this many bytes is pinned by the runtime for the copy (PCIe DMA rate); one of at most this many is
 * staged through the runtime's buffer by a CPU memcpy.  Host-tier calls with blocks above 256 KiB copy the
 * caller's pageable blocks directly, so this decides their speed: an RS(10,4) 1 MiB encode takes ~333 us
 * at threshold 0 and 478-596 us at the default ("Proxy environment").  The runtime reads
 * the variable once, when HIP initialises: set it in the process's launch environment.  -1 if the
 * variable is set but not a non-negative integer (the runtime's own parse then decides). */
long long ecg_host_pinned_xfer_threshold(void);

/* Kernel tuning options (process-wide; defaults also settable through the environment variables
 * ECG_NT, ECG_COLS_PER_WG, ECG_GRID_MAP, ECG_ZEROCOPY_BYTES, ECG_PROGRAM_CACHE, ECG_MAP_GROUP,
 * ECG_LAT_DWORD_BYTES, ECG_CALL_WORKER, ECG_ROW_SPLIT, ECG_GRAVEYARD, ECG_MT1_LDS_PAD).  Results never
 * depend on them. */
#define ECG_OPT_NT 0           /* non-temporal policy: bit 0 = loads, bit 1 = stores (default 3) */
#define ECG_OPT_COLS_PER_WG 1  /* 16-byte columns per workgroup, multiple of 128; 0 = auto (128 = 2 KiB) */
#define ECG_OPT_GRID_MAP 2     /* 0 = linear, 1 = XCD-contiguous, 2 = stripe s on XCD group s%8,
                                  3 = auto (default): 1 when outputs live inside the input stripes, else 2 */
#define ECG_OPT_ZEROCOPY_BYTES 3 /* host-buffer calls whose staged blocks total at most this many bytes
                                    run the kernel on mapped pinned memory (no DMA) and complete by
                                    polled flags; 0 = never; default 8 MiB (every staged call: blocks of
                                    at most 256 KiB) */
#define ECG_OPT_PROGRAM_CACHE 4 /* coefficient-table programs kept in HBM per device (LRU); when full, all
                                   but the newest half are dropped (retired: freed once the launches that
                                   used them completed, by per-stream events, never a device synchronize).
                                   Default 4096 */
#define ECG_OPT_MAP_GROUP 5    /* grid map 2: adjacent stripes per XCD group run (default 1 = stripe s on
                                  group s % 8); reduced to a power-of-two divisor tiling S when needed */
#define ECG_OPT_LAT_DWORD_BYTES 6 /* single calls (one stripe: host tier, or the device tier outside a batch
                                     scope) with blocks of at most this many bytes run the latency kernel:
                                     4 bytes per lane, every input load in flight at once; 0 = never;
                                     default 1 MiB (profiles/r02/lat_kernel/) */
#define ECG_OPT_CALL_WORKER 7 /* 0 = off (default); N > 0 = small synchronous host-tier calls (one op, <= 16
                                 inputs, <= 4 outputs, blocks of at most 16 KiB, 4-byte multiples) go to a
                                 resident kernel that polls a descriptor ring instead of launching one
                                 kernel per call, and that kernel exits after N us without a call.  RS(6,4)
                                 1 KiB: ~5 us instead of ~11 us per call.  The worker runs on a
                                 high-priority stream: leave it off in a process that runs its own work on
                                 high-priority streams */
#define ECG_OPT_ROW_SPLIT 8 /* batched launches whose op's output rows read disjoint input sets of one size,
                               with at least this many inputs in all (default 16; 0 = never), run each
                               (stripe, row) as its own launch stripe reading only that row's inputs: a
                               PC merge's 40 -> 5 XOR as five 8 -> 1 programs (fewer concurrent block
                               streams per workgroup; profiles/r04/pc_merge/) */
#define ECG_OPT_GRAVEYARD 9 /* evicted program sets allowed to wait for a stream the library is not handed
                               again (a destroyed or idle caller stream) before one device synchronize
                               frees them all (default 16384; >= 1; see ecg_program_sets_retiring) */
#define ECG_OPT_MT1_LDS_PAD 10 /* bytes of (unused) LDS reserved per workgroup of single-output vector launches
                                  (decode of one block, repairs, merges, XOR sums): caps how many of their
                                  workgroups share a CU.  -1 = by input count (default: 12-24 KiB, 2-6 %
                                  faster for 8-16 inputs, profiles/r05/occupancy/); 0 = no cap; else that
                                  many bytes, at most 65536.  Two-output launches take a fixed cap by input
                                  count (20-24 KiB from 8 inputs), and BINARY launches of 8-9 outputs 20 KiB
                                  from 12 inputs (profiles/r06/families/shape_probe/) */
#define ECG_OPT_COUNT 11
int ecg_set_option(int option, long long value);
long long ecg_get_option(int option);

/* ---------------------------------------------------------------- tier 1: Jerasure-compatible (w = 8)
 * Replaces reed_sol_vandermonde_coding_matrix  (called rs.cpp:7,34,297; lrc.cpp:624,935,1170) */
int* ecg_reed_sol_vandermonde_coding_matrix(int k, int m, int w);
/* Replaces cauchy_good_general_coding_matrix   (called lrc.cpp:1487,1522,1576,2099,2160,2215).
 * Returns NULL for m == 2 (cbest_8 path: unpinned). */
int* ecg_cauchy_good_general_coding_matrix(int k, int m, int w);
int* ecg_cauchy_original_coding_matrix(int k, int m, int w);
void ecg_cauchy_improve_coding_matrix(int k, int m, int w, int* matrix);
int ecg_cauchy_n_ones(int n, int w);
/* Replaces jerasure_invert_matrix              (called erasure_code.cpp:128; lrc.cpp:...) */
int ecg_jerasure_invert_matrix(int* mat, int* inv, int rows, int w);
/* Replaces jerasure_matrix_multiply            (called erasure_code.cpp:131; lrc.cpp:969,1203,1558,2197) */
int* ecg_jerasure_matrix_multiply(int* m1, int* m2, int r1, int c1, int r2, int c2, int w);
/* Replaces galois_region_xor(src, dest, nbytes): dest ^= src (host buffers).  Regions above 4096 bytes
 * (block data) are computed on the GPU.  Up to 4096 bytes -- what the reference's own calls pass: the
 * int coefficient rows of its Cauchy-LRC matrix builders, lrc.cpp:1511,2140 -- it is host matrix
 * construction and runs in place on the CPU, with no GPU round trip. */
int ecg_galois_region_xor(char* src, char* dest, int nbytes);
/* Replaces jerasure_matrix_encode              (called rs.cpp:24; lrc.cpp:28; erasure_code.cpp:90,109,147) */
int ecg_jerasure_matrix_encode(int k, int m, int w, int* matrix, char** data_ptrs, char** coding_ptrs, int size);
/* jerasure_matrix_dotprod (internal to a1/a3 in the reference): one row of k
 * coefficients into block dest_id (< k: data_ptrs[dest_id], else coding_ptrs[dest_id - k]); sources
 * are data_ptrs[0..k-1], or src_ids[i] in the same numbering.  An all-zero row leaves dest untouched.
 * ECG_EINVAL if dest is one of its own (nonzero-coefficient) sources. */
int ecg_jerasure_matrix_dotprod(int k, int w, int* matrix_row, int* src_ids, int dest_id, char** data_ptrs,
                                char** coding_ptrs, int size);
/* Replaces jerasure_matrix_decode              (called rs.cpp:36; lrc.cpp:50,66).  0 or -1 like the library. */
int ecg_jerasure_matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures, char** data_ptrs,
                               char** coding_ptrs, int size);

/* Host-side decode planning (SURVEY.md §8(b) "ecg_make_decode_matrix"): the whole of
 * jerasure_matrix_decode(k, m, matrix, row_k_ones, erasures) composed into ONE linear map.  Written
 * block dst_ids[i] = XOR_j coef[i * n_src + j] * block src_ids[j], block ids data 0..k-1 and coding
 * k..k+m-1, destinations in the library's write order.  Returns 0 with *n_src / *n_dst set (the arrays
 * are written only when cap_src >= *n_src and cap_dst >= *n_dst; coef needs *n_dst * *n_src ints),
 * ECG_EUNDECODABLE where the library returns -1, or ECG_EINVAL (bad arguments, or a pattern whose
 * library order reads a block after writing it, which has no single-map form). */
int ecg_make_decode_matrix(int k, int m, const int* matrix, int row_k_ones, const int* erasures, int* src_ids,
                           int cap_src, int* n_src, int* dst_ids, int cap_dst, int* n_dst, int* coef);

/* ---------------------------------------------------------------- tier 2: device / batched
 * All pointers below are DEVICE pointers; `stream` is a hipStream_t (NULL = default stream);
 * calls are asynchronous.  Block pointers must be 16-byte aligned for the vector path (otherwise a
 * byte path runs).  B is any byte count.  An empty batch (S == 0 or B == 0) is a no-op returning 0;
 * negative S or B is ECG_EINVAL. */
int ecg_dev_matrix_encode(int k, int m, const int* matrix, char** d_data_ptrs, char** d_coding_ptrs, long long B,
                          void* stream);
int ecg_dev_matrix_decode(int k, int m, const int* matrix, int row_k_ones, const int* erasures, char** d_data_ptrs,
                          char** d_coding_ptrs, long long B, void* stream);
/* Deferred-batch scope of the calling thread.  The reference issues one call per stripe
 * (proxy.cpp:312-349); on HBM-resident blocks each such call is a separate small launch, bound by
 * launch cost (~8 us per RS(10,4) call).  Between ecg_batch_begin() and ecg_batch_end(), device-tier
 * calls of this thread (ecg_dev_matrix_* and ErasureCode handles in ECG_MEM_DEVICE mode) are only
 * validated and recorded; ecg_batch_end() (or ecg_batch_flush()) launches them asynchronously on
 * their streams.  Recorded calls with the same plan, block size, stream and device are grouped into
 * ONE launch per op unless a data dependence orders them apart (a call reads or writes a block an
 * earlier call writes, or writes one an earlier call reads), so a per-stripe loop that interleaves
 * several plans -- a repair's helper partial, main partial and perform_addition per stripe -- still
 * goes out as one launch per plan.  Groups launch in an order that keeps every such dependence, across
 * streams too (where consecutive groups run on different streams, the later one's stream waits for an
 * event behind the earlier group): the outputs are the outputs of the calls run one by one in recorded
 * order, defined once the flush's work completes on their streams.  A group is a strided launch when its blocks are one strided batch (block b of the c-th call
 * at base + c * stripe_stride + b * block_stride, checked for every pointer), a pointer-table launch
 * otherwise.  Blocks are compared by address: blocks of one scope are identical or disjoint.
 * Host-tier and batched calls made inside the scope (ecg_region_xor_batch and ecg_fill_random
 * included) flush first.  A group launches on the device its calls were recorded on, whatever the
 * thread's device at flush time.  If a launch fails, the flush returns its error and the calls of that
 * group and of all later groups are discarded (the scope stays open, empty).  Scopes do not nest
 * (ECG_EINVAL).  While no scratch is declared (ecg_batch_scratch), the scope also flushes by itself
 * every 1024 recorded calls, so the GPU runs the first calls while the host records the rest; with
 * scratch declared, only every 65536 calls.  Declare scratch before recording the calls it is for.
 * Streams: a stream named by a recorded call must stay alive until the flush that launches the call
 * (the launch goes onto it).  After a flush returns, the library does not name its streams again, so a
 * caller may destroy them at once (ordering into the next flush uses an event recorded before return). */
int ecg_batch_begin(void);
int ecg_batch_flush(void);
int ecg_batch_end(void);
/* Inside a scope (ECG_EINVAL outside one): on = 1 defers HOST-tier calls of this thread too -- the
 * Jerasure-level calls and ErasureCode handles in ECG_MEM_HOST mode with blocks of at most 256 KiB.  Such a
 * call copies its input blocks into pinned staging when it is made (the caller may reuse them at once) and
 * writes its output blocks when the scope flushes: at ecg_batch_flush() / ecg_batch_end(), when a later
 * call of the scope reads or writes one of its output blocks (or uses another block size), when a
 * device-tier or batched call is made, and when the staging reaches 64 MiB.  Until then the caller must
 * not read those outputs.  A flush moves all staged inputs in one H2D copy, launches the calls grouped by
 * plan and moves the outputs back in one D2H copy: the per-call launch and completion round trip of a
 * synchronous host call (~10 us at 1 KiB, config 1's RS(6,4)) is paid once per flush.  Calls with larger
 * blocks run synchronously, as outside a scope.  on = 0 flushes the deferred host calls and stops
 * deferring; the flag resets at ecg_batch_begin. */
int ecg_batch_defer_host(int on);
/* Declare the device range [ptr, ptr + bytes) SCRATCH in the calling thread's scope (ECG_EINVAL outside
 * one).  The declaration holds until the scope ends and applies to every recorded call not yet flushed,
 * whether recorded before or after it.  A recorded call that writes a block inside scratch memory does
 * not write it: the flush keeps the linear combination the block would hold, and later recorded calls
 * that read the block read that combination's blocks instead.  So a partial result that only feeds a later call
 * of the scope -- a helper or main proxy's partial decode (erasure_code.cpp:113-150) consumed by
 * perform_addition (erasure_code.cpp:70-94) on the same GPU, handle_repair.cpp:249,371-376 -- costs no
 * HBM write and re-read.  The combination is written for real when it must be: before a block it reads
 * is overwritten, when it is read on another stream, device or block size, and at a mid-scope flush
 * (ecg_batch_flush(), a host-tier or batched call inside the scope, or the automatic flush every 65536
 * recorded calls).  After ecg_batch_end() the contents of scratch memory are undefined. */
int ecg_batch_scratch(const void* ptr, size_t bytes);
/* What this thread's last flush did: calls recorded, calls after scratch composition, launches (groups
 * x ops), scratch combinations written for real.  Any pointer may be NULL. */
int ecg_batch_last_stats(long long* recorded, long long* composed, long long* launches, long long* materialised);
/* Process-wide counters since the library loaded (diagnostics, every thread and device): region-product
 * kernels launched, and the bytes they move as planned -- a launch of S stripes over B-byte blocks whose op
 * reads k blocks and writes m, in row tiles that each read all k inputs, moves S * B * (tiles * k + m).  The
 * difference over a region of calls is the traffic those calls executed (bench.py's executed bytes; PMC
 * FETCH/WRITE counters agree where measured).  Either pointer may be NULL. */
int ecg_traffic_counters(long long* launches, long long* bytes);
/* Generic region product: out[dst_ids[p]] = XOR_j coef[p*k_in+j] * in[src_ids[j]] for S stripes,
 * in block b of stripe s at in_base + s*in_sstride + b*in_bstride (likewise out). */
int ecg_matrix_apply_batch(int k_in, int m_out, const int* coef, const int* src_ids, const int* dst_ids,
                           const void* in_base, long long in_sstride, long long in_bstride, void* out_base,
                           long long out_sstride, long long out_bstride, long long B, int S, void* stream);
/* Several programs in one launch (all k_in x m_out): launch stripe i runs program d_prog_of_stripe[i]
 * (device int[S]; NULL if n_prog == 1) on stripe d_stripe_of[i] (device int[S]; NULL = i) of the
 * strided layout.  coefs: n_prog x m_out x k_in; src_ids: n_prog x k_in; dst_ids: n_prog x m_out.
 * Used for rotating repair patterns (config 3) and for launching over a subset of a batch. */
int ecg_matrix_apply_batch_multi(int n_prog, int k_in, int m_out, const int* coefs, const int* src_ids,
                                 const int* dst_ids, const int* d_prog_of_stripe, const int* d_stripe_of,
                                 const void* in_base, long long in_sstride, long long in_bstride, void* out_base,
                                 long long out_sstride, long long out_bstride, long long B, int S, void* stream);
/* Batched jerasure_matrix_encode: in [S] x k blocks, out [S] x m blocks (coding block i at index i). */
int ecg_encode_batch(int k, int m, const int* matrix, const void* d_in, long long in_sstride, long long in_bstride,
                     void* d_out, long long out_sstride, long long out_bstride, long long B, int S, void* stream);
/* Batched jerasure_matrix_decode over stripes laid out as k+m blocks (data 0..k-1, coding k..k+m-1).
 * `patterns`: n_patterns host erasure lists, each -1-terminated, concatenated.  d_pattern_of_stripe:
 * device int[S] (NULL if n_patterns == 1).  Every pattern must compose to the same number of read
 * and written blocks.  d_out == NULL: written in place into the erased blocks; otherwise written
 * block i of a stripe's pattern (library write order) goes to d_out + s*out_sstride + i*out_bstride. */
int ecg_decode_batch(int k, int m, const int* matrix, int row_k_ones, const int* patterns, int n_patterns,
                     const int* d_pattern_of_stripe, void* d_stripes, long long sstride, long long bstride,
                     void* d_out, long long out_sstride, long long out_bstride, long long B, int S, void* stream);
/* Batched galois_region_xor: dst_s ^= src_s for S regions of nbytes (DEVICE pointers), region s at
 * d_src + s * src_stride and d_dst + s * dst_stride. */
int ecg_region_xor_batch(const void* d_src, long long src_stride, void* d_dst, long long dst_stride,
                         long long nbytes, int S, void* stream);
/* Batched perform_addition (erasure_code.cpp:70-94): parity i of stripe s = XOR_j partial[j*parity_num+i]. */
int ecg_perform_addition_batch(int block_num, int parity_num, const void* d_in, long long in_sstride,
                               long long in_bstride, void* d_out, long long out_sstride, long long out_bstride,
                               long long B, int S, void* stream);
/* Host-resident batches (the path starts and ends in host memory: proxy sockets / datanode buffers).
 * Same layouts as above but HOST pointers (pin them -- hipHostMalloc / hipHostRegister -- for full PCIe
 * rate).  Chunks of chunk_stripes stripes (0 = 16) flow through a 3-stage pipeline: H2D of the blocks
 * the program reads, kernel, D2H of the blocks it writes, on three streams so the three overlap.
 * Synchronous: returns when every output byte is in host memory. */
int ecg_encode_batch_host(int k, int m, const int* matrix, const void* h_in, long long in_sstride,
                          long long in_bstride, void* h_out, long long out_sstride, long long out_bstride, long long B,
                          int S, int chunk_stripes);
/* One erasure pattern for every stripe; h_out == NULL writes the rebuilt blocks in place. */
int ecg_decode_batch_host(int k, int m, const int* matrix, int row_k_ones, const int* erasures, void* h_stripes,
                          long long sstride, long long bstride, void* h_out, long long out_sstride,
                          long long out_bstride, long long B, int S, int chunk_stripes);
/* Deterministic synthetic bytes (splitmix64 counter). */
int ecg_fill_random(void* d_dst, long long nbytes, unsigned long long seed, unsigned long long word_offset,
                    void* stream);

/* ---------------------------------------------------------------- tier 3: ErasureCode facade */
enum ecg_ectype {  /* project/include/ec/erasure_code.h:17-29 */
    ECG_RS = 0,
    ECG_ERS = 1,
    ECG_AZURE_LRC = 2,
    ECG_AZURE_LRC_1 = 3,
    ECG_OPTIMAL_LRC = 4,
    ECG_OPTIMAL_CAUCHY_LRC = 5,
    ECG_UNIFORM_CAUCHY_LRC = 6,
    ECG_PC = 7,
    ECG_HIERACHICAL_PC = 8,
    ECG_HV_PC = 9
};

typedef struct ecg_coding_parameters {  /* erasure_code.h:38-51 */
    int k, m, l, g, k1, m1, k2, m2, x, seri_num;
    int local_or_column;
} ecg_coding_parameters;

#define ECG_MEM_HOST 0   /* char** point at host buffers (reference semantics, synchronous) */
#define ECG_MEM_DEVICE 1 /* char** point at HBM buffers, asynchronous on the handle's stream */

typedef struct ecg_ec ecg_ec;

ecg_ec* ecg_ec_factory(int ec_type, const ecg_coding_parameters* cp); /* metadata.cpp:48-77 */
void ecg_ec_destroy(ecg_ec* ec);
int ecg_ec_init_coding_parameters(ecg_ec* ec, const ecg_coding_parameters* cp);
int ecg_ec_get_coding_parameters(ecg_ec* ec, ecg_coding_parameters* cp);
/* ECG_MEM_DEVICE: later calls on the handle launch on `stream`.  The handle stores it, so the stream must
 * stay alive while the handle's calls use it; the library itself never names it after a call returns
 * (evicted program sets are retired without it; see ecg_program_sets_retiring). */
int ecg_ec_set_memory(ecg_ec* ec, int mem, void* stream);
int ecg_ec_set_isvertical(ecg_ec* ec, int isvertical); /* HPC::isvertical (pc.h:66) */
int ecg_ec_k(const ecg_ec* ec);
int ecg_ec_m(const ecg_ec* ec);
int ecg_ec_make_encoding_matrix(ecg_ec* ec, int* final_matrix); /* m x k, where the class defines one */
int ecg_ec_check_if_decodable(ecg_ec* ec, const int* failure_idxs, int n);
int ecg_ec_encode(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size);
int ecg_ec_decode(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num);
int ecg_ec_encode_partial_blocks_for_encoding(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size,
                                              const int* data_idxs, int n_data, const int* parity_idxs,
                                              int n_parity);
int ecg_ec_encode_partial_blocks_for_decoding(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size,
                                              const int* local_survivor_idxs, int n_local,
                                              const int* survivor_idxs, int n_survivors,
                                              const int* failure_idxs, int n_failures);
int ecg_ec_perform_addition(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size, int block_num,
                            int parity_num);
/* The main proxy's end of a partial-decoding repair (handle_repair.cpp:371-376: its own
 * encode_partial_blocks_for_decoding over local_ptrs, then perform_addition with the helpers' partials)
 * in ONE pass: out[u] = partial_u(local blocks) XOR (XOR_j partial_ptrs[j*n_failures + u]).  Same bytes
 * as the two calls, without writing and re-reading the main proxy's own partials.  n_local may be 0
 * (pure addition); n_partials must be a multiple of n_failures. */
int ecg_ec_encode_partial_blocks_for_decoding_with_addition(ecg_ec* ec, char** local_ptrs, char** partial_ptrs,
                                                            int n_partials, char** out_ptrs, int block_size,
                                                            const int* local_survivor_idxs, int n_local,
                                                            const int* survivor_idxs, int n_survivors,
                                                            const int* failure_idxs, int n_failures);
/* Stripe-merging counterpart (handle_merge.cpp:159,319): the parity proxy's own
 * encode_partial_blocks_for_encoding over local_ptrs plus perform_addition of the helpers' partial
 * parities, in one pass.  n_data may be 0; n_partials must be a multiple of n_parity. */
int ecg_ec_encode_partial_blocks_for_encoding_with_addition(ecg_ec* ec, char** local_ptrs, char** partial_ptrs,
                                                            int n_partials, char** out_ptrs, int block_size,
                                                            const int* data_idxs, int n_data, const int* parity_idxs,
                                                            int n_parity);
/* Planning hooks for batching: the coefficient matrix (n_out x n_in, row-major) that the facade's
 * partial call would apply to its data_ptrs -> coding_ptrs.  Returns n_out (>= 0) or a negative code;
 * feed the result to ecg_matrix_apply_batch. */
int ecg_ec_partial_decoding_matrix(ecg_ec* ec, const int* local_survivor_idxs, int n_local,
                                   const int* survivor_idxs, int n_survivors, const int* failure_idxs,
                                   int n_failures, int* out_coef, int out_cap);
int ecg_ec_partial_encoding_matrix(ecg_ec* ec, const int* data_idxs, int n_data, const int* parity_idxs,
                                   int n_parity, int* out_coef, int out_cap);

/* ---- partitioning and repair planning (host logic) ----
 * Placement rules: erasure_code.h:31-36 PlacementRule, plus Azu_LRC::partition_sub_optimal
 * (lrc.cpp:816-873), which the reference defines but never reaches from generate_partition. */
#define ECG_PLACE_FLAT 0
#define ECG_PLACE_RANDOM 1
#define ECG_PLACE_OPTIMAL 2     /* the reference's default (erasure_code.h:66) */
#define ECG_PLACE_SUB_OPTIMAL 3 /* Azure LRC only */
int ecg_ec_set_placement_rule(ecg_ec* ec, int rule);
/* Seed of the per-object stream behind RANDOM placement (default: std::random_device). */
int ecg_ec_set_random_seed(ecg_ec* ec, unsigned long long seed);
/* ErasureCode::generate_partition (erasure_code.cpp:159-169). */
int ecg_ec_generate_partition(ecg_ec* ec);
/* The current partition_plan, serialised as [n_partitions, (size, block ids...)*].  Returns the number
 * of ints the encoding needs; `buf` is written only when cap >= that number. */
int ecg_ec_get_partition(ecg_ec* ec, int* buf, int cap);
/* Overwrite partition_plan (same encoding as ecg_ec_get_partition), as the coordinator does from the
 * actual block placement before planning a repair (auxs.cpp:139-159). */
int ecg_ec_set_partition(ecg_ec* ec, const int* buf, int len);
/* LRC grouping_information (lrc.h:73): [n_groups, (size, block ids...)*]; ECG_EINVAL for other codes. */
int ecg_ec_grouping_information(ecg_ec* ec, int* buf, int cap);
/* ErasureCode::generate_repair_plan (rs.cpp:264-279, lrc.cpp:445-574 / 1861-2023, pc.cpp:451-551 /
 * 1166-1264) over the current partition_plan.  *decodable = 1 (plans made) or 0 (undecodable; the
 * reference's false).  Plans serialised as [n_plans, (local_or_column, n_failures, ids...,
 * n_help, (size, ids...)*)*].  Returns the number of ints needed (written when cap suffices) or < 0. */
int ecg_ec_generate_repair_plan(ecg_ec* ec, const int* failure_idxs, int n, int* buf, int cap, int* decodable);
/* Block-index helpers the coordinator and proxies use.  LRC (lrc.h:67-71): group of a block, its index in
 * the group's encoding space, group size (+ first block id).  Product codes (pc.h:44-45): grid position.
 * ECG_EINVAL when the code has no such notion. */
int ecg_ec_bid2gid(ecg_ec* ec, int block_id);
int ecg_ec_idxingroup(ecg_ec* ec, int block_id);
int ecg_ec_get_group_size(ecg_ec* ec, int group_id, int* min_idx);
int ecg_ec_bid2rowcol(ecg_ec* ec, int block_id, int* row, int* col);
int ecg_ec_rowcol2bid(ecg_ec* ec, int row, int col);
/* ErasureCode::self_information (e.g. "RS(10,4)"); returns the length, writes when cap > length. */
int ecg_ec_self_information(ecg_ec* ec, char* buf, int cap);

#ifdef __cplusplus
}
#endif
#endif /* ECG_H */
