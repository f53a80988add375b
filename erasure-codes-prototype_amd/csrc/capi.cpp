// extern "C" entry points declared in include/ecg.h.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/ecg.h"
#include "codes.hpp"
#include "engine.hpp"

using namespace ecg;

struct ecg_ec {
    ErasureCode* impl;
};

namespace {

int* to_malloc(const std::vector<int>& v) {
    if (v.empty()) return nullptr;
    int* p = (int*)malloc(v.size() * sizeof(int));
    if (p) memcpy(p, v.data(), v.size() * sizeof(int));
    return p;
}

std::vector<int> vec(const int* p, int n) { return n > 0 && p ? std::vector<int>(p, p + n) : std::vector<int>(); }

void put_lists(std::vector<int>& out, const std::vector<std::vector<int>>& lists) {
    out.push_back((int)lists.size());
    for (auto& l : lists) {
        out.push_back((int)l.size());
        out.insert(out.end(), l.begin(), l.end());
    }
}

int emit(const std::vector<int>& v, int* buf, int cap) {
    if (buf && cap >= (int)v.size()) memcpy(buf, v.data(), v.size() * sizeof(int));
    return (int)v.size();
}

}  // namespace

extern "C" {

const char* ecg_last_error(void) { return last_error_string(); }
int ecg_version(void) { return 101; }  // 1.1: batch scope, fused repair/merge calls, decode-matrix export

int ecg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ecg_set_device(int device) { return hipSetDevice(device) == hipSuccess ? ECG_OK : ECG_EHIP; }

void ecg_free(void* p) { free(p); }

int ecg_program_cache_size(void) { return (int)Engine::instance().cache_size(); }
int ecg_program_sets_retiring(void) { return (int)Engine::instance().retired_pending(); }
int ecg_program_sets_reclaim(void) { return (int)Engine::instance().reclaim(); }
int ecg_host_contexts(void) { return Engine::instance().host_contexts(); }

int ecg_call_worker_stats(long long* calls, long long* launches, long long* relaunches, int* disabled) {
    return call_worker_stats(calls, launches, relaunches, disabled);
}

long long ecg_host_pinned_xfer_threshold(void) {
    const char* v = getenv("GPU_PINNED_MIN_XFER_SIZE");
    if (!v || !*v) return 1LL << 20;  // the runtime's default: 1 MiB
    char* end = nullptr;
    const long long mib = strtoll(v, &end, 10);
    if (*end != '\0' || mib < 0 || mib > (1LL << 40)) return -1;
    return mib << 20;
}

int ecg_batch_begin(void) { return batch_begin(); }
int ecg_batch_flush(void) { return batch_flush_all(); }
int ecg_batch_defer_host(int on) { return batch_defer_host(on); }
int ecg_batch_end(void) { return batch_end(); }
int ecg_batch_scratch(const void* ptr, size_t bytes) { return batch_scratch(ptr, bytes); }
int ecg_batch_last_stats(long long* recorded, long long* composed, long long* launches, long long* materialised) {
    const FlushStats s = last_flush_stats();
    if (recorded) *recorded = s.recorded;
    if (composed) *composed = s.composed;
    if (launches) *launches = s.launches;
    if (materialised) *materialised = s.materialised;
    return ECG_OK;
}

int ecg_traffic_counters(long long* launches, long long* bytes) {
    launch_traffic(launches, bytes);
    return ECG_OK;
}

int ecg_set_option(int option, long long value) { return set_option(option, value) == 0 ? ECG_OK : ECG_EINVAL; }
long long ecg_get_option(int option) { return get_option(option); }

// ------------------------------------------------------------------------------ tier 1

int* ecg_reed_sol_vandermonde_coding_matrix(int k, int m, int w) {
    if (w != 8) return nullptr;
    return to_malloc(reed_sol_vandermonde_coding_matrix(k, m));
}

int* ecg_cauchy_good_general_coding_matrix(int k, int m, int w) {
    if (w != 8) return nullptr;
    return to_malloc(cauchy_good_general_coding_matrix(k, m));
}

int* ecg_cauchy_original_coding_matrix(int k, int m, int w) {
    if (w != 8) return nullptr;
    return to_malloc(cauchy_original_coding_matrix(k, m));
}

void ecg_cauchy_improve_coding_matrix(int k, int m, int w, int* matrix) {
    if (w != 8 || !matrix || k < 1 || m < 1) return;
    std::vector<int> M(matrix, matrix + (size_t)k * m);
    cauchy_improve_coding_matrix(k, m, M);
    memcpy(matrix, M.data(), M.size() * sizeof(int));
}

int ecg_cauchy_n_ones(int n, int w) { return w == 8 ? cauchy_n_ones(n) : -1; }

int ecg_jerasure_invert_matrix(int* mat, int* inv, int rows, int w) {
    if (w != 8 || rows < 1 || !mat || !inv) return -1;
    std::vector<int> a(mat, mat + (size_t)rows * rows), b;
    const int rc = invert_matrix(a, b, rows);
    memcpy(mat, a.data(), a.size() * sizeof(int));  // the library works in place on `mat`
    memcpy(inv, b.data(), b.size() * sizeof(int));
    return rc;
}

int* ecg_jerasure_matrix_multiply(int* m1, int* m2, int r1, int c1, int r2, int c2, int w) {
    // Jerasure indexes m2 as c1 x c2 without checking c1 == r2; a mismatch is refused here
    if (w != 8 || !m1 || !m2 || r1 < 1 || c1 < 1 || c2 < 1 || c1 != r2) return nullptr;
    return to_malloc(matrix_multiply(m1, m2, r1, c1, r2, c2));
}

// The reference calls galois_region_xor itself only inside its Cauchy-LRC matrix builders, to add the
// global rows' int coefficients into a local row (lrc.cpp:1511,2140: 4 * k bytes of host matrix), and
// rebuilds those matrices on every call (lrc.cpp:27).  Regions up to kHostXorMax bytes are that matrix
// work (host-side, keep on CPU) and are XORed in place here; a GPU round trip
// (~15 us) per coefficient row would cost more than the whole encode of a small stripe.  Larger
// regions -- block data -- run on the GPU like every other region product.
constexpr int kHostXorMax = 4096;

int ecg_galois_region_xor(char* src, char* dest, int nbytes) {
    if (nbytes < 0 || !src || !dest) return ECG_EINVAL;
    if (nbytes <= kHostXorMax) {
        if (const int rc = batch_flush_pending(); rc != ECG_OK) return rc;  // host-tier call order, as run_host
        for (int i = 0; i < nbytes; i++) dest[i] ^= src[i];
        return ECG_OK;
    }
    LinearOp op;
    op.src_ids = {0, 1};
    op.dst_ids = {1};
    op.coef = {1, 1};
    uint8_t* blocks[2] = {(uint8_t*)src, (uint8_t*)dest};
    return Engine::instance().run_host({op}, blocks, 2, nbytes);
}

int ecg_jerasure_matrix_encode(int k, int m, int w, int* matrix, char** data_ptrs, char** coding_ptrs, int size) {
    if (w != 8 || k < 1 || m < 1 || !matrix || !data_ptrs || !coding_ptrs || size < 0) return ECG_EINVAL;
    const auto plan = encode_plan_cached(k, m, matrix);
    if (plan->empty()) return ECG_OK;
    thread_local std::vector<uint8_t*> blocks;
    blocks.resize((size_t)k + m);
    for (int i = 0; i < k; i++) blocks[i] = (uint8_t*)data_ptrs[i];
    for (int i = 0; i < m; i++) blocks[(size_t)k + i] = (uint8_t*)coding_ptrs[i];
    return Engine::instance().run_host(*plan, blocks.data(), k + m, size);
}

int ecg_jerasure_matrix_dotprod(int k, int w, int* matrix_row, int* src_ids, int dest_id, char** data_ptrs,
                                char** coding_ptrs, int size) {
    if (w != 8 || k < 1 || !matrix_row || dest_id < 0 || size < 0) return ECG_EINVAL;
    int max_id = dest_id;
    LinearOp op;
    for (int i = 0; i < k; i++) {
        const int c = matrix_row[i];
        if (c < 0 || c > 255) return ECG_EINVAL;
        const int id = src_ids ? src_ids[i] : i;
        if (id < 0) return ECG_EINVAL;
        if (c == 0) continue;
        op.src_ids.push_back(id);
        op.coef.push_back((uint8_t)c);
        max_id = std::max(max_id, id);
    }
    if (op.src_ids.empty()) return ECG_OK;  // all-zero row: destination untouched
    // dest among its own sources: Jerasure's in-place sequential update would depend on term order;
    // the reference never asks for it (destinations are coding or erased blocks), so refuse it
    if (std::find(op.src_ids.begin(), op.src_ids.end(), dest_id) != op.src_ids.end()) return ECG_EINVAL;
    op.dst_ids.push_back(dest_id);
    std::vector<uint8_t*> blocks((size_t)max_id + 1, nullptr);
    for (int id = 0; id <= max_id; id++) {
        char** base = id < k ? data_ptrs : coding_ptrs;
        blocks[id] = base ? (uint8_t*)base[id < k ? id : id - k] : nullptr;
    }
    return Engine::instance().run_host({op}, blocks.data(), max_id + 1, size);
}

int ecg_jerasure_matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures, char** data_ptrs,
                               char** coding_ptrs, int size) {
    if (w != 8 || k < 1 || m < 1 || !matrix || !erasures || !data_ptrs || !coding_ptrs || size < 0) return -1;
    std::vector<LinearOp> ops;
    if (plan_matrix_decode(k, m, matrix, row_k_ones, erasures, ops) < 0) return -1;
    std::vector<uint8_t*> blocks((size_t)k + m);
    for (int i = 0; i < k; i++) blocks[i] = (uint8_t*)data_ptrs[i];
    for (int i = 0; i < m; i++) blocks[(size_t)k + i] = (uint8_t*)coding_ptrs[i];
    const int rc = Engine::instance().run_host(ops, blocks.data(), k + m, size);
    return rc == ECG_OK ? 0 : rc;
}

// ------------------------------------------------------------------------------ tier 2

int ecg_dev_matrix_encode(int k, int m, const int* matrix, char** d_data_ptrs, char** d_coding_ptrs, long long B,
                          void* stream) {
    if (k < 1 || m < 1 || !matrix || !d_data_ptrs || !d_coding_ptrs || B < 0) return ECG_EINVAL;
    LinearOp op = plan_matrix_encode(k, m, matrix);
    if (op.m_out() == 0) return ECG_OK;
    std::vector<uint8_t*> blocks((size_t)k + m);
    for (int i = 0; i < k; i++) blocks[i] = (uint8_t*)d_data_ptrs[i];
    for (int i = 0; i < m; i++) blocks[(size_t)k + i] = (uint8_t*)d_coding_ptrs[i];
    return Engine::instance().run_device({op}, blocks.data(), k + m, B, (hipStream_t)stream);
}

int ecg_dev_matrix_decode(int k, int m, const int* matrix, int row_k_ones, const int* erasures, char** d_data_ptrs,
                          char** d_coding_ptrs, long long B, void* stream) {
    if (k < 1 || m < 1 || !matrix || !erasures || !d_data_ptrs || !d_coding_ptrs || B < 0) return ECG_EINVAL;
    std::vector<LinearOp> ops;
    if (plan_matrix_decode(k, m, matrix, row_k_ones, erasures, ops) < 0) return ECG_EUNDECODABLE;
    std::vector<uint8_t*> blocks((size_t)k + m);
    for (int i = 0; i < k; i++) blocks[i] = (uint8_t*)d_data_ptrs[i];
    for (int i = 0; i < m; i++) blocks[(size_t)k + i] = (uint8_t*)d_coding_ptrs[i];
    return Engine::instance().run_device(ops, blocks.data(), k + m, B, (hipStream_t)stream);
}

int ecg_matrix_apply_batch(int k_in, int m_out, const int* coef, const int* src_ids, const int* dst_ids,
                           const void* in_base, long long in_sstride, long long in_bstride, void* out_base,
                           long long out_sstride, long long out_bstride, long long B, int S, void* stream) {
    if (k_in < 1 || m_out < 1 || !coef || !src_ids || !dst_ids) return ECG_EINVAL;
    LinearOp op;
    op.src_ids = vec(src_ids, k_in);
    op.dst_ids = vec(dst_ids, m_out);
    op.coef.resize((size_t)k_in * m_out);
    for (size_t i = 0; i < op.coef.size(); i++) op.coef[i] = (uint8_t)(coef[i] & 0xff);
    return Engine::instance().run_strided({op}, nullptr, S, in_base, in_sstride, in_bstride, out_base, out_sstride,
                                          out_bstride, B, (hipStream_t)stream);
}

int ecg_matrix_apply_batch_multi(int n_prog, int k_in, int m_out, const int* coefs, const int* src_ids,
                                 const int* dst_ids, const int* d_prog_of_stripe, const int* d_stripe_of,
                                 const void* in_base, long long in_sstride, long long in_bstride, void* out_base,
                                 long long out_sstride, long long out_bstride, long long B, int S, void* stream) {
    if (n_prog < 1 || k_in < 1 || m_out < 1 || !coefs || !src_ids || !dst_ids) return ECG_EINVAL;
    if (n_prog > 1 && !d_prog_of_stripe) return ECG_EINVAL;
    std::vector<LinearOp> progs(n_prog);
    for (int p = 0; p < n_prog; p++) {
        LinearOp& op = progs[p];
        op.src_ids = vec(src_ids + (size_t)p * k_in, k_in);
        op.dst_ids = vec(dst_ids + (size_t)p * m_out, m_out);
        op.coef.resize((size_t)k_in * m_out);
        const int* c = coefs + (size_t)p * k_in * m_out;
        for (size_t i = 0; i < op.coef.size(); i++) op.coef[i] = (uint8_t)(c[i] & 0xff);
    }
    return Engine::instance().run_strided(progs, d_prog_of_stripe, S, in_base, in_sstride, in_bstride, out_base,
                                          out_sstride, out_bstride, B, (hipStream_t)stream, d_stripe_of);
}

int ecg_encode_batch(int k, int m, const int* matrix, const void* d_in, long long in_sstride, long long in_bstride,
                     void* d_out, long long out_sstride, long long out_bstride, long long B, int S, void* stream) {
    if (k < 1 || m < 1 || !matrix) return ECG_EINVAL;
    LinearOp op = plan_matrix_encode(k, m, matrix);
    if (op.m_out() == 0) return ECG_OK;
    for (int& d : op.dst_ids) d -= k;  // coding block i -> out block i
    return Engine::instance().run_strided({op}, nullptr, S, d_in, in_sstride, in_bstride, d_out, out_sstride,
                                          out_bstride, B, (hipStream_t)stream);
}

int ecg_decode_batch(int k, int m, const int* matrix, int row_k_ones, const int* patterns, int n_patterns,
                     const int* d_pattern_of_stripe, void* d_stripes, long long sstride, long long bstride,
                     void* d_out, long long out_sstride, long long out_bstride, long long B, int S, void* stream) {
    if (k < 1 || m < 1 || !matrix || !patterns || n_patterns < 1) return ECG_EINVAL;
    if (n_patterns > 1 && !d_pattern_of_stripe) return ECG_EINVAL;
    std::vector<LinearOp> progs;
    const int* pat = patterns;
    for (int p = 0; p < n_patterns; p++) {
        std::vector<LinearOp> ops;
        if (plan_matrix_decode(k, m, matrix, row_k_ones, pat, ops) < 0) return ECG_EUNDECODABLE;
        if (ops.size() != 1) return ECG_EINVAL;  // non-composable pattern: use ecg_dev_matrix_decode
        if (d_out)
            for (size_t i = 0; i < ops[0].dst_ids.size(); i++) ops[0].dst_ids[i] = (int)i;
        if (!progs.empty() && (ops[0].k_in() != progs[0].k_in() || ops[0].m_out() != progs[0].m_out()))
            return ECG_EINVAL;
        progs.push_back(std::move(ops[0]));
        while (*pat != -1) pat++;
        pat++;
    }
    void* out = d_out ? d_out : d_stripes;
    return Engine::instance().run_strided(progs, d_pattern_of_stripe, S, d_stripes, sstride, bstride, out,
                                          d_out ? out_sstride : sstride, d_out ? out_bstride : bstride, B,
                                          (hipStream_t)stream);
}

int ecg_encode_batch_host(int k, int m, const int* matrix, const void* h_in, long long in_sstride,
                          long long in_bstride, void* h_out, long long out_sstride, long long out_bstride, long long B,
                          int S, int chunk_stripes) {
    if (k < 1 || m < 1 || !matrix) return ECG_EINVAL;
    LinearOp op = plan_matrix_encode(k, m, matrix);
    if (op.m_out() == 0) return ECG_OK;
    for (int& d : op.dst_ids) d -= k;
    return Engine::instance().run_host_pipeline(op, h_in, in_sstride, in_bstride, h_out, out_sstride, out_bstride, B,
                                                S, chunk_stripes);
}

int ecg_decode_batch_host(int k, int m, const int* matrix, int row_k_ones, const int* erasures, void* h_stripes,
                          long long sstride, long long bstride, void* h_out, long long out_sstride,
                          long long out_bstride, long long B, int S, int chunk_stripes) {
    if (k < 1 || m < 1 || !matrix || !erasures) return ECG_EINVAL;
    std::vector<LinearOp> ops;
    if (plan_matrix_decode(k, m, matrix, row_k_ones, erasures, ops) < 0) return ECG_EUNDECODABLE;
    if (ops.empty()) return ECG_OK;
    if (ops.size() != 1) return ECG_EINVAL;
    if (h_out)
        for (size_t i = 0; i < ops[0].dst_ids.size(); i++) ops[0].dst_ids[i] = (int)i;
    return Engine::instance().run_host_pipeline(ops[0], h_stripes, sstride, bstride, h_out ? h_out : h_stripes,
                                                h_out ? out_sstride : sstride, h_out ? out_bstride : bstride, B, S,
                                                chunk_stripes);
}

int ecg_make_decode_matrix(int k, int m, const int* matrix, int row_k_ones, const int* erasures, int* src_ids,
                           int cap_src, int* n_src, int* dst_ids, int cap_dst, int* n_dst, int* coef) {
    if (k < 1 || m < 1 || !matrix || !erasures || !n_src || !n_dst) return ECG_EINVAL;
    std::vector<LinearOp> ops;
    if (plan_matrix_decode(k, m, matrix, row_k_ones, erasures, ops) < 0) return ECG_EUNDECODABLE;
    if (ops.size() > 1) return ECG_EINVAL;
    const LinearOp empty;
    const LinearOp& op = ops.empty() ? empty : ops[0];
    *n_src = op.k_in();
    *n_dst = op.m_out();
    if (cap_src >= op.k_in() && cap_dst >= op.m_out() && src_ids && dst_ids && coef) {
        std::copy(op.src_ids.begin(), op.src_ids.end(), src_ids);
        std::copy(op.dst_ids.begin(), op.dst_ids.end(), dst_ids);
        for (size_t i = 0; i < op.coef.size(); i++) coef[i] = op.coef[i];
    }
    return ECG_OK;
}

int ecg_region_xor_batch(const void* d_src, long long src_stride, void* d_dst, long long dst_stride,
                         long long nbytes, int S, void* stream) {
    if (S < 0 || nbytes < 0) return ECG_EINVAL;
    if (S == 0 || nbytes == 0) return ECG_OK;
    if (!d_src || !d_dst) return ECG_EINVAL;
    // recorded calls of an open batch scope go first (the pointer-table launch below does not flush)
    if (const int rc = batch_flush_pending(); rc != ECG_OK) return rc;
    LinearOp op;
    op.src_ids = {0, 1};
    op.dst_ids = {1};
    op.coef = {1, 1};
    std::vector<std::vector<const uint8_t*>> blk((size_t)S);
    std::vector<const uint8_t* const*> calls((size_t)S);
    for (int s = 0; s < S; s++) {
        blk[s] = {(const uint8_t*)d_src + (size_t)s * src_stride, (const uint8_t*)d_dst + (size_t)s * dst_stride};
        calls[s] = blk[s].data();
    }
    Engine& e = Engine::instance();
    bool done = false;  // regular strides (the usual case): the strided launch, else a pointer table
    const int rc = e.run_calls_strided(op, calls, nbytes, (hipStream_t)stream, &done);
    return done || rc != ECG_OK ? rc : e.run_ptr_batch(op, calls, nbytes, (hipStream_t)stream);
}

int ecg_perform_addition_batch(int block_num, int parity_num, const void* d_in, long long in_sstride,
                               long long in_bstride, void* d_out, long long out_sstride, long long out_bstride,
                               long long B, int S, void* stream) {
    if (parity_num < 1 || block_num < 1 || block_num % parity_num != 0) return ECG_EINVAL;
    LinearOp op;
    for (int j = 0; j < block_num; j++) op.src_ids.push_back(j);
    for (int i = 0; i < parity_num; i++) op.dst_ids.push_back(i);
    op.coef.assign((size_t)block_num * parity_num, 0);
    for (int i = 0; i < parity_num; i++)
        for (int j = 0; j < block_num / parity_num; j++) op.coef[(size_t)i * block_num + j * parity_num + i] = 1;
    return Engine::instance().run_strided({op}, nullptr, S, d_in, in_sstride, in_bstride, d_out, out_sstride,
                                          out_bstride, B, (hipStream_t)stream);
}

int ecg_fill_random(void* d_dst, long long nbytes, unsigned long long seed, unsigned long long word_offset,
                    void* stream) {
    if (!d_dst || nbytes < 0) return ECG_EINVAL;
    if (const int rc = batch_flush_pending(); rc != ECG_OK) return rc;
    hipError_t e = launch_fill_splitmix(d_dst, nbytes, seed, word_offset, (hipStream_t)stream);
    if (e != hipSuccess) {
        set_last_error(std::string("fill: ") + hipGetErrorString(e));
        return ECG_EHIP;
    }
    return ECG_OK;
}

// ------------------------------------------------------------------------------ tier 3

ecg_ec* ecg_ec_factory(int ec_type, const ecg_coding_parameters* cp) {
    if (!cp) return nullptr;
    ErasureCode* impl = ec_factory(ec_type, *cp);
    if (!impl) return nullptr;
    return new ecg_ec{impl};
}

void ecg_ec_destroy(ecg_ec* ec) {
    if (!ec) return;
    delete ec->impl;
    delete ec;
}

int ecg_ec_init_coding_parameters(ecg_ec* ec, const ecg_coding_parameters* cp) {
    if (!ec || !cp) return ECG_EINVAL;
    ec->impl->init_coding_parameters(*cp);
    return ECG_OK;
}

int ecg_ec_get_coding_parameters(ecg_ec* ec, ecg_coding_parameters* cp) {
    if (!ec || !cp) return ECG_EINVAL;
    ec->impl->get_coding_parameters(*cp);
    return ECG_OK;
}

int ecg_ec_set_memory(ecg_ec* ec, int mem, void* stream) {
    if (!ec || (mem != ECG_MEM_HOST && mem != ECG_MEM_DEVICE)) return ECG_EINVAL;
    ec->impl->mem = mem;
    ec->impl->stream = (hipStream_t)stream;
    return ECG_OK;
}

int ecg_ec_set_isvertical(ecg_ec* ec, int isvertical) {
    if (!ec) return ECG_EINVAL;
    HPC* h = dynamic_cast<HPC*>(ec->impl);
    if (!h) return ECG_EINVAL;
    h->isvertical = isvertical != 0;
    return ECG_OK;
}

int ecg_ec_k(const ecg_ec* ec) { return ec ? ec->impl->k : ECG_EINVAL; }
int ecg_ec_m(const ecg_ec* ec) { return ec ? ec->impl->m : ECG_EINVAL; }

int ecg_ec_make_encoding_matrix(ecg_ec* ec, int* final_matrix) {
    if (!ec || !final_matrix) return ECG_EINVAL;
    return ec->impl->make_encoding_matrix(final_matrix);
}

int ecg_ec_check_if_decodable(ecg_ec* ec, const int* failure_idxs, int n) {
    if (!ec || n < 0) return ECG_EINVAL;
    return ec->impl->check_if_decodable(vec(failure_idxs, n));
}

int ecg_ec_encode(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size) {
    if (!ec || !data_ptrs || !coding_ptrs || block_size < 0) return ECG_EINVAL;
    return ec->impl->encode(data_ptrs, coding_ptrs, block_size);
}

int ecg_ec_decode(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) {
    if (!ec || !data_ptrs || !coding_ptrs || !erasures || block_size < 0 || failed_num < 0) return ECG_EINVAL;
    return ec->impl->decode(data_ptrs, coding_ptrs, block_size, erasures, failed_num);
}

int ecg_ec_encode_partial_blocks_for_encoding(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size,
                                              const int* data_idxs, int n_data, const int* parity_idxs,
                                              int n_parity) {
    if (!ec || n_data < 1 || n_parity < 1 || block_size < 0) return ECG_EINVAL;
    return ec->impl->encode_partial_blocks_for_encoding(data_ptrs, coding_ptrs, block_size, vec(data_idxs, n_data),
                                                        vec(parity_idxs, n_parity));
}

int ecg_ec_encode_partial_blocks_for_decoding(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size,
                                              const int* local_survivor_idxs, int n_local,
                                              const int* survivor_idxs, int n_survivors,
                                              const int* failure_idxs, int n_failures) {
    if (!ec || n_local < 1 || n_survivors < 1 || n_failures < 1 || block_size < 0) return ECG_EINVAL;
    return ec->impl->encode_partial_blocks_for_decoding(data_ptrs, coding_ptrs, block_size,
                                                        vec(local_survivor_idxs, n_local),
                                                        vec(survivor_idxs, n_survivors),
                                                        vec(failure_idxs, n_failures));
}

int ecg_ec_encode_partial_blocks_for_decoding_with_addition(ecg_ec* ec, char** local_ptrs, char** partial_ptrs,
                                                            int n_partials, char** out_ptrs, int block_size,
                                                            const int* local_survivor_idxs, int n_local,
                                                            const int* survivor_idxs, int n_survivors,
                                                            const int* failure_idxs, int n_failures) {
    if (!ec || !out_ptrs || n_local < 0 || n_partials < 0 || n_failures < 1 || block_size < 0) return ECG_EINVAL;
    if ((n_local > 0 && (!local_ptrs || !local_survivor_idxs || !survivor_idxs || n_survivors < 1)) ||
        (n_partials > 0 && !partial_ptrs) || !failure_idxs)
        return ECG_EINVAL;
    return ec->impl->encode_partial_blocks_for_decoding_with_addition(
        local_ptrs, partial_ptrs, n_partials, out_ptrs, block_size, vec(local_survivor_idxs, n_local),
        vec(survivor_idxs, n_survivors), vec(failure_idxs, n_failures));
}

int ecg_ec_encode_partial_blocks_for_encoding_with_addition(ecg_ec* ec, char** local_ptrs, char** partial_ptrs,
                                                            int n_partials, char** out_ptrs, int block_size,
                                                            const int* data_idxs, int n_data, const int* parity_idxs,
                                                            int n_parity) {
    if (!ec || !out_ptrs || n_data < 0 || n_partials < 0 || n_parity < 1 || !parity_idxs || block_size < 0)
        return ECG_EINVAL;
    if ((n_data > 0 && (!local_ptrs || !data_idxs)) || (n_partials > 0 && !partial_ptrs)) return ECG_EINVAL;
    return ec->impl->encode_partial_blocks_for_encoding_with_addition(local_ptrs, partial_ptrs, n_partials, out_ptrs,
                                                                      block_size, vec(data_idxs, n_data),
                                                                      vec(parity_idxs, n_parity));
}

int ecg_ec_perform_addition(ecg_ec* ec, char** data_ptrs, char** coding_ptrs, int block_size, int block_num,
                            int parity_num) {
    if (!ec || block_size < 0) return ECG_EINVAL;
    return ec->impl->perform_addition(data_ptrs, coding_ptrs, block_size, block_num, parity_num);
}

int ecg_ec_partial_decoding_matrix(ecg_ec* ec, const int* local_survivor_idxs, int n_local,
                                   const int* survivor_idxs, int n_survivors, const int* failure_idxs,
                                   int n_failures, int* out_coef, int out_cap) {
    if (!ec || !out_coef) return ECG_EINVAL;
    std::vector<int> M;
    int rc = ec->impl->partial_decoding_matrix(vec(local_survivor_idxs, n_local), vec(survivor_idxs, n_survivors),
                                               vec(failure_idxs, n_failures), M);
    if (rc != ECG_OK) return rc;
    if ((int)M.size() > out_cap) return ECG_EINVAL;
    memcpy(out_coef, M.data(), M.size() * sizeof(int));
    return n_failures;
}

int ecg_ec_partial_encoding_matrix(ecg_ec* ec, const int* data_idxs, int n_data, const int* parity_idxs,
                                   int n_parity, int* out_coef, int out_cap) {
    if (!ec || !out_coef) return ECG_EINVAL;
    std::vector<int> M;
    int rc = ec->impl->partial_encoding_matrix(vec(data_idxs, n_data), vec(parity_idxs, n_parity), M);
    if (rc != ECG_OK) return rc;
    if ((int)M.size() > out_cap) return ECG_EINVAL;
    memcpy(out_coef, M.data(), M.size() * sizeof(int));
    return n_parity;
}

// ---- partitioning and repair planning (planning.cpp)

int ecg_ec_set_placement_rule(ecg_ec* ec, int rule) {
    if (!ec || rule < ECG_PLACE_FLAT || rule > ECG_PLACE_SUB_OPTIMAL) return ECG_EINVAL;
    ec->impl->placement_rule = rule;
    return ECG_OK;
}

int ecg_ec_set_random_seed(ecg_ec* ec, unsigned long long seed) {
    if (!ec) return ECG_EINVAL;
    ec->impl->set_random_seed(seed);
    return ECG_OK;
}

int ecg_ec_generate_partition(ecg_ec* ec) {
    if (!ec) return ECG_EINVAL;
    return ec->impl->generate_partition();
}

int ecg_ec_get_partition(ecg_ec* ec, int* buf, int cap) {
    if (!ec || cap < 0) return ECG_EINVAL;
    std::vector<int> out;
    put_lists(out, ec->impl->partition_plan);
    return emit(out, buf, cap);
}

int ecg_ec_set_partition(ecg_ec* ec, const int* buf, int len) {
    if (!ec || !buf || len < 1) return ECG_EINVAL;
    const int n_blocks = ec->impl->k + ec->impl->m;
    std::vector<std::vector<int>> plan;
    int at = 1;
    for (int p = 0; p < buf[0]; p++) {
        if (at >= len) return ECG_EINVAL;
        const int sz = buf[at++];
        if (sz < 0 || at + sz > len) return ECG_EINVAL;
        std::vector<int> part(buf + at, buf + at + sz);
        for (int b : part)
            if (b < 0 || b >= n_blocks) return ECG_EINVAL;
        plan.push_back(part);
        at += sz;
    }
    ec->impl->partition_plan = plan;
    return ECG_OK;
}

int ecg_ec_grouping_information(ecg_ec* ec, int* buf, int cap) {
    if (!ec || cap < 0) return ECG_EINVAL;
    auto* lrc = dynamic_cast<LocallyRepairableCode*>(ec->impl);
    if (!lrc) return ECG_EINVAL;
    std::vector<std::vector<int>> groups;
    lrc->grouping_information(groups);
    std::vector<int> out;
    put_lists(out, groups);
    return emit(out, buf, cap);
}

int ecg_ec_generate_repair_plan(ecg_ec* ec, const int* failure_idxs, int n, int* buf, int cap, int* decodable) {
    if (!ec || n <= 0 || !failure_idxs || cap < 0) return ECG_EINVAL;
    std::vector<RepairPlan> plans;
    const int rc = ec->impl->generate_repair_plan(vec(failure_idxs, n), plans);
    if (rc < 0) return rc;
    if (decodable) *decodable = rc;
    std::vector<int> out;
    out.push_back((int)plans.size());
    for (auto& p : plans) {
        out.push_back(p.local_or_column ? 1 : 0);
        out.push_back((int)p.failure_idxs.size());
        out.insert(out.end(), p.failure_idxs.begin(), p.failure_idxs.end());
        put_lists(out, p.help_blocks);
    }
    return emit(out, buf, cap);
}

int ecg_ec_bid2gid(ecg_ec* ec, int block_id) {
    auto* lrc = ec ? dynamic_cast<LocallyRepairableCode*>(ec->impl) : nullptr;
    if (!lrc || block_id < 0 || block_id >= lrc->k + lrc->m) return ECG_EINVAL;
    return lrc->bid2gid(block_id);
}

int ecg_ec_idxingroup(ecg_ec* ec, int block_id) {
    auto* lrc = ec ? dynamic_cast<LocallyRepairableCode*>(ec->impl) : nullptr;
    if (!lrc || block_id < 0 || block_id >= lrc->k + lrc->m) return ECG_EINVAL;
    return lrc->idxingroup(block_id);
}

int ecg_ec_get_group_size(ecg_ec* ec, int group_id, int* min_idx) {
    auto* lrc = ec ? dynamic_cast<LocallyRepairableCode*>(ec->impl) : nullptr;
    if (!lrc || group_id < 0 || group_id > lrc->l) return ECG_EINVAL;
    int mi = 0;
    const int gs = lrc->get_group_size(group_id, mi);
    if (min_idx) *min_idx = mi;
    return gs;
}

int ecg_ec_bid2rowcol(ecg_ec* ec, int block_id, int* row, int* col) {
    auto* pc = ec ? dynamic_cast<ProductCode*>(ec->impl) : nullptr;
    if (!pc || !row || !col || block_id < 0 || block_id >= pc->k + pc->m) return ECG_EINVAL;
    pc->bid2rowcol(block_id, *row, *col);
    return ECG_OK;
}

int ecg_ec_rowcol2bid(ecg_ec* ec, int row, int col) {
    auto* pc = ec ? dynamic_cast<ProductCode*>(ec->impl) : nullptr;
    if (!pc || row < 0 || col < 0 || row >= pc->k2 + pc->m2 || col >= pc->k1 + pc->m1) return ECG_EINVAL;
    return pc->rowcol2bid(row, col);
}

int ecg_ec_self_information(ecg_ec* ec, char* buf, int cap) {
    if (!ec || cap < 0) return ECG_EINVAL;
    const std::string s = ec->impl->self_information();
    if (buf && cap > (int)s.size()) memcpy(buf, s.c_str(), s.size() + 1);
    return (int)s.size();
}

}  // extern "C"
