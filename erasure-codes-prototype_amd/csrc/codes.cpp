// ErasureCode facade implementation.  Each method cites the reference lines it mirrors
// (paths relative to /root/reference/project).
#include "codes.hpp"

#include <string.h>

#include <algorithm>
#include <typeinfo>

#include "engine.hpp"
#include "gf256.hpp"
#include "gf_kernels.hpp"

namespace ecg {

// ================================================================================== plan helpers

static void remap(LinearOp& op, int k, const std::vector<int>& data_ids, const std::vector<int>& coding_ids) {
    auto f = [&](int id) { return id < k ? data_ids[id] : coding_ids[id - k]; };
    for (int& id : op.src_ids) id = f(id);
    for (int& id : op.dst_ids) id = f(id);
}

void append_encode(Plan& plan, int k, int m, const int* matrix, const std::vector<int>& data_ids,
                   const std::vector<int>& coding_ids) {
    LinearOp op = plan_matrix_encode(k, m, matrix);
    if (op.m_out() == 0) return;
    remap(op, k, data_ids, coding_ids);
    plan.ops.push_back(std::move(op));
}

int append_decode(Plan& plan, int k, int m, const int* matrix, int row_k_ones, const int* erasures,
                  const std::vector<int>& data_ids, const std::vector<int>& coding_ids) {
    std::vector<LinearOp> ops;
    if (plan_matrix_decode(k, m, matrix, row_k_ones, erasures, ops) < 0) return ECG_EUNDECODABLE;
    for (LinearOp& op : ops) {
        remap(op, k, data_ids, coding_ids);
        plan.ops.push_back(std::move(op));
    }
    return ECG_OK;
}

static std::vector<int> iota_ids(int n, int base = 0) {
    std::vector<int> v(n);
    for (int i = 0; i < n; i++) v[i] = base + i;
    return v;
}

// ================================================================================== ErasureCode

void ErasureCode::init_coding_parameters(const CodingParameters& cp) {  // erasure_code.cpp:5-10
    k = cp.k;
    m = cp.m;
    local_or_column = cp.local_or_column != 0;
}

void ErasureCode::get_coding_parameters(CodingParameters& cp) const {  // erasure_code.cpp:12-17
    cp.k = k;
    cp.m = m;
    cp.local_or_column = local_or_column;
}

namespace {

uint64_t hash_ints(const std::vector<int>& v) {
    uint64_t h = 1469598103934665603ull;
    for (int x : v) h = (h ^ (uint32_t)x) * 1099511628211ull;
    return h;
}

template <class V>
class KeyedCache {
public:
    const V* find(const std::vector<int>& key, uint64_t h) const {
        auto it = map_.find(h);
        if (it == map_.end()) return nullptr;
        for (auto& e : it->second)
            if (e.first == key) return &e.second;
        return nullptr;
    }
    const V& put(std::vector<int> key, uint64_t h, V v) {
        if (++n_ > kMax) {
            map_.clear();
            n_ = 1;
        }
        auto& bucket = map_[h];
        bucket.emplace_back(std::move(key), std::move(v));
        return bucket.back().second;
    }

private:
    static constexpr size_t kMax = 1024;
    std::unordered_map<uint64_t, std::vector<std::pair<std::vector<int>, V>>> map_;
    size_t n_ = 0;
};

}  // namespace

void ErasureCode::state_key(std::vector<int>& key) const {
    const size_t t = typeid(*this).hash_code();
    key.insert(key.end(), {(int)(uint32_t)t, (int)(uint32_t)((uint64_t)t >> 32), k, m, w, (int)local_or_column});
}

void EnlargedRSCode::state_key(std::vector<int>& key) const {
    RSCode::state_key(key);
    key.insert(key.end(), {x, seri_num});
}

void LocallyRepairableCode::state_key(std::vector<int>& key) const {
    ErasureCode::state_key(key);
    key.insert(key.end(), {l, g, r});
}

void ProductCode::state_key(std::vector<int>& key) const {
    ErasureCode::state_key(key);
    key.insert(key.end(), {k1, m1, k2, m2});
    row_code.state_key(key);
    col_code.state_key(key);
}

void HPC::state_key(std::vector<int>& key) const {
    ProductCode::state_key(key);
    key.push_back((int)isvertical);
    e_row_code.state_key(key);
    e_col_code.state_key(key);
}

void ErasureCode::get_full_matrix(int* matrix, int kk) {  // erasure_code.cpp:30-35
    for (int i = 0; i < kk; i++) matrix[(size_t)i * kk + i] = 1;
}

void ErasureCode::make_submatrix_by_rows(int cols, const int* matrix, int* new_matrix,
                                         const std::vector<int>& idxs) {  // erasure_code.cpp:37-47
    for (size_t i = 0; i < idxs.size(); i++)
        memcpy(&new_matrix[i * cols], &matrix[(size_t)idxs[i] * cols], (size_t)cols * sizeof(int));
}

void ErasureCode::make_submatrix_by_cols(int cols, int rows, const int* matrix, int* new_matrix,
                                         const std::vector<int>& idxs) {  // erasure_code.cpp:49-61
    const int n = (int)idxs.size();
    for (int i = 0; i < n; i++)
        for (int u = 0; u < rows; u++) new_matrix[(size_t)u * n + i] = matrix[(size_t)u * cols + idxs[i]];
}

// erasure_code.cpp:97-111 (the matrix handed to jerasure_matrix_encode)
void ErasureCode::partial_encoding_matrix_(int k_, const int* full, const std::vector<int>& data_idxs,
                                           const std::vector<int>& parity_idxs, std::vector<int>& out) {
    const int nb = (int)data_idxs.size(), np = (int)parity_idxs.size();
    std::vector<int> rows((size_t)np * k_, 0);
    make_submatrix_by_rows(k_, full, rows.data(), parity_idxs);
    out.assign((size_t)np * nb, 1);
    make_submatrix_by_cols(k_, np, rows.data(), out.data(), data_idxs);
}

// erasure_code.cpp:113-150: R = F[failures] * inv(F[survivors]); columns of the local survivors.
void ErasureCode::partial_decoding_matrix_(int k_, const int* full, const std::vector<int>& lsi,
                                           const std::vector<int>& si, const std::vector<int>& fi,
                                           std::vector<int>& out) {
    const int nl = (int)lsi.size(), nf = (int)fi.size();
    // memo keyed by everything the result depends on: the ids and the rows of `full` they select
    thread_local KeyedCache<std::vector<int>> memo;
    thread_local std::vector<int> key;
    const size_t ns = si.size(), len = 4 + (size_t)nl + ns + (size_t)nf + (ns + (size_t)nf) * (size_t)k_;
    key.resize(len);
    int* w = key.data();
    *w++ = k_;
    *w++ = nl;
    *w++ = (int)ns;
    *w++ = nf;
    for (int x : lsi) *w++ = x;
    for (int x : si) *w++ = x;
    for (int x : fi) *w++ = x;
    for (int r : si) w = std::copy(full + (size_t)r * k_, full + (size_t)r * k_ + k_, w);
    for (int r : fi) w = std::copy(full + (size_t)r * k_, full + (size_t)r * k_ + k_, w);
    const uint64_t h = hash_ints(key);
    if (const std::vector<int>* hit = memo.find(key, h)) {
        out = *hit;
        return;
    }
    std::vector<int> fm((size_t)nf * k_, 0), sm((size_t)k_ * k_, 0), inv;
    make_submatrix_by_rows(k_, full, fm.data(), fi);
    make_submatrix_by_rows(k_, full, sm.data(), si);
    (void)invert_matrix(sm, inv, k_);  // return value ignored, erasure_code.cpp:128
    std::vector<int> dec = matrix_multiply(fm.data(), inv.data(), nf, k_, k_, k_);
    out.assign((size_t)nf * nl, 0);
    for (int i = 0; i < nl; i++) {
        int idx = 0;
        for (int s : si) {
            if (s == lsi[i]) break;
            idx++;
        }
        for (int u = 0; u < nf; u++) {
            const size_t at = (size_t)u * k_ + idx;
            out[(size_t)u * nl + i] = at < dec.size() ? dec[at] : 0;
        }
    }
    memo.put(key, h, out);
}

namespace {

// Per-thread plan caches.  The proxy makes one ErasureCode call per stripe (proxy.cpp:312-349,
// handle_repair.cpp:249,375), and a batch scope records such a call in ~0.1 us, so rebuilding the
// call's coefficient matrix (a Gauss-Jordan inversion per partial decode, erasure_code.cpp:113-150) and
// its plan each time would dominate.  Keys are the exact inputs of the computation (ids and matrix
// entries), so a hit is the value the computation would return; each cache is bounded and simply
// cleared when full.
// jerasure_matrix_encode(kk, mm, matrix) as an interned plan (matrix.hpp)
SharedOps encode_plan(int kk, int mm, const int* matrix) { return encode_plan_cached(kk, mm, matrix); }

}  // namespace

int ErasureCode::run(const SharedOps& ops, char** data_ptrs, int n_data, char** coding_ptrs, int n_coding,
                     long long B) {
    if (ops->empty()) return ECG_OK;
    const int n = n_data + n_coding;
    uint8_t* small[64];
    std::vector<uint8_t*> large;
    uint8_t** blocks = small;
    if (n > 64) {
        large.resize((size_t)n);
        blocks = large.data();
    }
    for (int i = 0; i < n_data; i++) blocks[i] = (uint8_t*)data_ptrs[i];
    for (int i = 0; i < n_coding; i++) blocks[n_data + i] = (uint8_t*)coding_ptrs[i];
    Engine& eng = Engine::instance();
    if (mem == ECG_MEM_DEVICE) return eng.run_device(ops, blocks, n, B, stream);
    return eng.run_host(*ops, blocks, n, B);
}

int ErasureCode::run(const Plan& plan, char** data_ptrs, int n_data, char** coding_ptrs, int n_coding,
                     long long B) {
    if (plan.ops.empty()) return ECG_OK;
    const int n = n_data + n_coding;
    uint8_t* small[64];  // the common case needs no allocation (per-stripe calls are launch-rate bound)
    std::vector<uint8_t*> large;
    uint8_t** blocks = small;
    if (n > 64) {
        large.resize((size_t)n);
        blocks = large.data();
    }
    for (int i = 0; i < n_data; i++) blocks[i] = (uint8_t*)data_ptrs[i];
    for (int i = 0; i < n_coding; i++) blocks[n_data + i] = (uint8_t*)coding_ptrs[i];
    Engine& eng = Engine::instance();
    if (mem == ECG_MEM_DEVICE) return eng.run_device(plan.ops, blocks, n, B, stream);
    return eng.run_host(plan.ops, blocks, n, B);
}

int ErasureCode::run_encode(int kk, int mm, const int* matrix, char** data_ptrs, char** coding_ptrs, long long B,
                            bool stable_matrix) {
    // The encode plan's block ids are already the call's (data 0..kk-1, coding kk..kk+mm-1).  A matrix
    // from the process-wide builder cache never changes behind its pointer, so its plan is reused by
    // pointer (one entry per thread); any other matrix goes through the content-keyed plan cache.
    if (stable_matrix) {
        thread_local const int* last_matrix = nullptr;
        thread_local int last_k = -1, last_m = -1;
        thread_local SharedOps last_plan;
        if (matrix != last_matrix || kk != last_k || mm != last_m) {
            last_plan = encode_plan(kk, mm, matrix);
            last_matrix = matrix;
            last_k = kk;
            last_m = mm;
        }
        return run(last_plan, data_ptrs, kk, coding_ptrs, mm, B);
    }
    return run(encode_plan(kk, mm, matrix), data_ptrs, kk, coding_ptrs, mm, B);
}

// ---- whole-call plans: composition and the per-thread plan cache
//
// A multi-step method (product-code encode: row codes, then column codes over data AND the row parities just
// written, pc.cpp:39-76; the iterative decodes, pc.cpp:79-195, 921-1029) plans one op per sub-code call.  Run
// as planned, each op is a launch and the column ops re-read the data and the parities the row ops wrote:
// PC(4,1,4,1) encode moves 45 blocks for 16 in and 9 out.  compose_chain substitutes every read of a block
// the call itself wrote with that block's expression over the call's inputs (exact, by linearity), so the
// call becomes ONE op that reads each input once and writes each output once (25 blocks, one launch).
// Blocks a row tile of the kernel moves: every tile reads all of its op's inputs.
static long long op_traffic(const LinearOp& op) {
    const int mt = op_is_binary(op) ? kMaxMTBin : kMaxMT;
    return (long long)(op.m_out() + mt - 1) / mt * op.k_in() + op.m_out();
}

// The chain as the engine should run it: composed when that moves no more blocks than the chain and, for the
// GENERAL flavour (straight-line dense fold, every coefficient of a tile folded even where it is 0), keeps the
// fold within 6 coefficient products per block moved -- RS(10,4)'s encode folds 40 per 14 blocks at ~35 % of
// gfx950's VALU issue at the HBM roofline (gf_kernels.hip header).  Otherwise the ops as planned.
static SharedOps finish_plan(std::vector<LinearOp>&& ops) {
    auto out = std::make_shared<std::vector<LinearOp>>();
    LinearOp one;
    if (ops.size() > 1 && compose_chain(ops, one)) {
        long long chained = 0;
        for (const LinearOp& op : ops) chained += op_traffic(op);
        const long long moved = op_traffic(one);
        const bool binary = op_is_binary(one);
        const long long tiles = (one.m_out() + kMaxMT - 1) / kMaxMT;
        const bool valu_ok = binary || (long long)one.k_in() * tiles * kMaxMT <= 6 * moved;
        if (moved <= chained && valu_ok) {
            out->push_back(std::move(one));
            return out;
        }
    }
    *out = std::move(ops);
    return out;
}

namespace {
struct CallPlan {
    SharedOps ops;
    int status = ECG_OK;  // the planner's status (an undecodable iterative decode still runs what it planned)
};
}  // namespace

static KeyedCache<CallPlan>& call_plans() {
    thread_local KeyedCache<CallPlan> cache;
    return cache;
}

// Find the plan of the call keyed by `key` -- the exact inputs of its planning -- or make it with build(plan),
// which returns the planner's status.  Returns that status; cp is set unless the status is an error other than
// ECG_EUNDECODABLE (nothing is cached or run then).  An undecodable iterative decode keeps the work it planned.
template <class Build>
static int run_planned(const std::vector<int>& key, Build build, const CallPlan*& cp) {
    const uint64_t h = hash_ints(key);
    cp = call_plans().find(key, h);
    if (cp) return cp->status;
    Plan p;
    const int status = build(p);
    if (status != ECG_OK && status != ECG_EUNDECODABLE) return status;
    cp = &call_plans().put(key, h, CallPlan{finish_plan(std::move(p.ops)), status});
    return status;
}

int ErasureCode::run_decode(int kk, int mm, const int* matrix, int row_k_ones, int* erasures, char** data_ptrs,
                            char** coding_ptrs, long long B) {
    // keyed by everything plan_matrix_decode reads: shape, flag, matrix entries, the -1-terminated erasures
    thread_local std::vector<int> key;
    key.assign({6, kk, mm, row_k_ones});
    key.insert(key.end(), matrix, matrix + (size_t)kk * mm);
    for (int i = 0; erasures[i] != -1; i++) key.push_back(erasures[i]);  // the planner reads up to the -1 too
    const CallPlan* cp = nullptr;
    const int rc = run_planned(key, [&](Plan& p) {
        return append_decode(p, kk, mm, matrix, row_k_ones, erasures, iota_ids(kk), iota_ids(mm, kk));
    }, cp);
    if (rc != ECG_OK) return rc;  // the library decodes nothing when it returns -1

    return run(cp->ops, data_ptrs, kk, coding_ptrs, mm, B);
}

// Per-thread cache of the partial calls' plans, keyed by the object's state_key and the call's index
// lists: a proxy repairing stripe after stripe repeats the same few patterns, and the matrix behind a
// partial decode is an inversion.
static KeyedCache<SharedOps>& partial_plans() {
    thread_local KeyedCache<SharedOps> cache;
    return cache;
}

static void append_list(std::vector<int>& key, const std::vector<int>& v) {
    key.push_back((int)v.size());
    key.insert(key.end(), v.begin(), v.end());
}

int ErasureCode::encode_partial_blocks_for_encoding(char** data_ptrs, char** coding_ptrs, int block_size,
                                                    std::vector<int> data_idxs, std::vector<int> parity_idxs) {
    const int nd = (int)data_idxs.size(), np = (int)parity_idxs.size();
    thread_local std::vector<int> key;
    key.assign({2});
    state_key(key);
    append_list(key, data_idxs);
    append_list(key, parity_idxs);
    const uint64_t h = hash_ints(key);
    if (const SharedOps* hit = partial_plans().find(key, h)) return run(*hit, data_ptrs, nd, coding_ptrs, np, block_size);
    std::vector<int> M;
    int rc = partial_encoding_matrix(std::move(data_idxs), std::move(parity_idxs), M);
    if (rc != ECG_OK) return rc;
    const SharedOps plan = partial_plans().put(key, h, encode_plan(nd, np, M.data()));
    return run(plan, data_ptrs, nd, coding_ptrs, np, block_size);
}

int ErasureCode::encode_partial_blocks_for_decoding(char** data_ptrs, char** coding_ptrs, int block_size,
                                                    std::vector<int> lsi, std::vector<int> si,
                                                    std::vector<int> fi) {
    const int nl = (int)lsi.size(), nf = (int)fi.size();
    thread_local std::vector<int> key;
    key.assign({3});
    state_key(key);
    append_list(key, lsi);
    append_list(key, si);
    append_list(key, fi);
    const uint64_t h = hash_ints(key);
    if (const SharedOps* hit = partial_plans().find(key, h)) return run(*hit, data_ptrs, nl, coding_ptrs, nf, block_size);
    std::vector<int> M;
    int rc = partial_decoding_matrix(std::move(lsi), std::move(si), std::move(fi), M);
    if (rc != ECG_OK) return rc;
    const SharedOps plan = partial_plans().put(key, h, encode_plan(nl, nf, M.data()));
    return run(plan, data_ptrs, nl, coding_ptrs, nf, block_size);
}

// erasure_code.cpp:70-94: coding[i] = XOR_j data[j * parity_num + i], one launch for all i.
int ErasureCode::perform_addition(char** data_ptrs, char** coding_ptrs, int block_size, int block_num,
                                  int parity_num) {
    if (parity_num <= 0 || block_num < 0 || block_num % parity_num != 0) return ECG_EINVAL;
    if (block_num == 0) return ECG_OK;
    thread_local KeyedCache<SharedOps> cache;
    std::vector<int> key{1, block_num, parity_num};
    const uint64_t h = hash_ints(key);
    const SharedOps* plan = cache.find(key, h);
    if (!plan) {
        LinearOp op;
        op.src_ids = iota_ids(block_num);
        op.dst_ids = iota_ids(parity_num, block_num);
        op.coef.assign((size_t)parity_num * block_num, 0);
        const int per = block_num / parity_num;
        for (int i = 0; i < parity_num; i++)
            for (int j = 0; j < per; j++) op.coef[(size_t)i * block_num + (size_t)j * parity_num + i] = 1;
        plan = &cache.put(std::move(key), h, std::make_shared<const std::vector<LinearOp>>(1, std::move(op)));
    }
    return run(*plan, data_ptrs, block_num, coding_ptrs, parity_num, block_size);
}

// out[u] = XOR_i R[u][i] * local[i]  XOR  XOR_j partial[j * nf + u]  (one launch)
int ErasureCode::run_with_addition(const std::vector<int>& R, int nl, int nf, char** local_ptrs,
                                   char** partial_ptrs, int n_partials, char** out_ptrs, long long B) {
    LinearOp op;
    const int n_in = nl + n_partials;
    op.src_ids = iota_ids(n_in);
    op.dst_ids = iota_ids(nf, n_in);
    op.coef.assign((size_t)nf * n_in, 0);
    for (int u = 0; u < nf; u++) {
        for (int i = 0; i < nl; i++) op.coef[(size_t)u * n_in + i] = R[(size_t)u * nl + i] & 0xff;
        for (int j = 0; j < n_partials / nf; j++) op.coef[(size_t)u * n_in + nl + (size_t)j * nf + u] = 1;
    }
    std::vector<char*> in((size_t)n_in);
    for (int i = 0; i < nl; i++) in[i] = local_ptrs[i];
    for (int j = 0; j < n_partials; j++) in[(size_t)nl + j] = partial_ptrs[j];
    Plan p;
    p.ops.push_back(std::move(op));
    return run(p, in.data(), n_in, out_ptrs, nf, B);
}

int ErasureCode::encode_partial_blocks_for_decoding_with_addition(char** local_ptrs, char** partial_ptrs,
                                                                  int n_partials, char** out_ptrs, int block_size,
                                                                  std::vector<int> lsi, std::vector<int> si,
                                                                  std::vector<int> fi) {
    const int nl = (int)lsi.size(), nf = (int)fi.size();
    if (nf < 1 || n_partials < 0 || n_partials % nf != 0 || block_size < 0) return ECG_EINVAL;
    if (nl + n_partials == 0) return ECG_EINVAL;
    std::vector<int> R;
    if (nl > 0) {
        int rc = partial_decoding_matrix(std::move(lsi), std::move(si), std::move(fi), R);
        if (rc != ECG_OK) return rc;
    }
    return run_with_addition(R, nl, nf, local_ptrs, partial_ptrs, n_partials, out_ptrs, block_size);
}

int ErasureCode::encode_partial_blocks_for_encoding_with_addition(char** local_ptrs, char** partial_ptrs,
                                                                  int n_partials, char** out_ptrs, int block_size,
                                                                  std::vector<int> data_idxs,
                                                                  std::vector<int> parity_idxs) {
    const int nl = (int)data_idxs.size(), nf = (int)parity_idxs.size();
    if (nf < 1 || n_partials < 0 || n_partials % nf != 0 || block_size < 0) return ECG_EINVAL;
    if (nl + n_partials == 0) return ECG_EINVAL;
    std::vector<int> R;
    if (nl > 0) {
        int rc = partial_encoding_matrix(std::move(data_idxs), std::move(parity_idxs), R);
        if (rc != ECG_OK) return rc;
    }
    return run_with_addition(R, nl, nf, local_ptrs, partial_ptrs, n_partials, out_ptrs, block_size);
}

static bool ids_in_range(const std::vector<int>& v, int n) {
    for (int x : v)
        if (x < 0 || x >= n) return false;
    return true;
}

// ================================================================================== RS / ERS

const std::vector<int>& RSCode::vandermonde() { return cached_vandermonde(k, m); }

int RSCode::make_encoding_matrix(int* final_matrix) {  // rs.cpp:5-18
    const std::vector<int>& v = vandermonde();
    if (v.empty()) return ECG_EINVAL;
    std::copy(v.begin(), v.end(), final_matrix);
    return ECG_OK;
}

std::vector<int> RSCode::full_matrix() {  // rs.cpp:48-50
    std::vector<int> f((size_t)(k + m) * k, 0);
    get_full_matrix(f.data(), k);
    make_encoding_matrix(&f[(size_t)k * k]);
    return f;
}

int RSCode::encode(char** data_ptrs, char** coding_ptrs, int block_size) {  // rs.cpp:20-25
    if (typeid(*this) != typeid(RSCode)) {  // EnlargedRSCode: its own make_encoding_matrix
        std::vector<int> M((size_t)k * m, 0);
        int rc = make_encoding_matrix(M.data());
        if (rc != ECG_OK) return rc;
        return run_encode(k, m, M.data(), data_ptrs, coding_ptrs, block_size);
    }
    const std::vector<int>& v = vandermonde();
    if (v.empty()) return ECG_EINVAL;
    return run_encode(k, m, v.data(), data_ptrs, coding_ptrs, block_size, /*stable_matrix=*/true);
}

// rs.cpp:27-42.  NB: decodes with reed_sol_vandermonde_coding_matrix(k, m) even for EnlargedRSCode,
// and passes failed_num as row_k_ones, exactly like the reference.
int RSCode::decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) {
    if (failed_num > m) return ECG_EUNDECODABLE;
    const std::vector<int>& v = vandermonde();
    if (v.empty()) return ECG_EINVAL;
    return run_decode(k, m, v.data(), failed_num, erasures, data_ptrs, coding_ptrs, block_size);
}

int RSCode::plan_encode(Plan& p, const std::vector<int>& data_ids, const std::vector<int>& coding_ids) {
    std::vector<int> M((size_t)k * m, 0);
    int rc = make_encoding_matrix(M.data());
    if (rc != ECG_OK) return rc;
    append_encode(p, k, m, M.data(), data_ids, coding_ids);
    return ECG_OK;
}

int RSCode::plan_decode(Plan& p, const std::vector<int>& data_ids, const std::vector<int>& coding_ids,
                        int* erasures, int failed_num) {
    if (failed_num > m) return ECG_EUNDECODABLE;
    const std::vector<int>& v = vandermonde();
    if (v.empty()) return ECG_EINVAL;
    return append_decode(p, k, m, v.data(), failed_num, erasures, data_ids, coding_ids);
}

int RSCode::check_if_decodable(const std::vector<int>& f) { return m >= (int)f.size() ? 1 : 0; }  // rs.cpp:68-76

int RSCode::partial_encoding_matrix(std::vector<int> data_idxs, std::vector<int> parity_idxs,
                                    std::vector<int>& out) {  // rs.cpp:44-53
    if (!ids_in_range(data_idxs, k) || !ids_in_range(parity_idxs, k + m)) return ECG_EINVAL;
    std::vector<int> f = full_matrix();
    partial_encoding_matrix_(k, f.data(), data_idxs, parity_idxs, out);
    return ECG_OK;
}

int RSCode::partial_decoding_matrix(std::vector<int> lsi, std::vector<int> si, std::vector<int> fi,
                                    std::vector<int>& out) {  // rs.cpp:55-66
    if ((int)si.size() > k || !ids_in_range(si, k + m) || !ids_in_range(fi, k + m)) return ECG_EINVAL;
    std::vector<int> f = full_matrix();
    partial_decoding_matrix_(k, f.data(), lsi, si, fi, out);
    return ECG_OK;
}

std::string RSCode::self_information() const {
    return "RS(" + std::to_string(k) + "," + std::to_string(m) + ")";
}

void EnlargedRSCode::init_coding_parameters(const CodingParameters& cp) {  // rs.cpp:282-288
    k = cp.k;
    m = cp.m;
    x = cp.x;
    seri_num = cp.seri_num;
}

int EnlargedRSCode::make_encoding_matrix(int* final_matrix) {  // rs.cpp:290-305
    if (seri_num >= x) return ECG_OK;  // "Invalid argurments!": the caller's zeros stay
    const std::vector<int>& big = cached_vandermonde(x * k, m);
    if (big.empty()) return ECG_EINVAL;
    for (int i = 0; i < m; i++)
        memcpy(&final_matrix[(size_t)i * k], &big[(size_t)i * k * x + (size_t)seri_num * k], (size_t)k * sizeof(int));
    return ECG_OK;
}

std::string EnlargedRSCode::self_information() const {
    return "EnlargedRS(" + std::to_string(k) + "," + std::to_string(m) + "|" + std::to_string(x) + "," +
           std::to_string(seri_num) + ")";
}

// ================================================================================== LRC base

void LocallyRepairableCode::init_coding_parameters(const CodingParameters& cp) {  // lrc.cpp:5-12
    k = cp.k;
    l = cp.l;
    g = cp.g;
    m = l + g;
    local_or_column = cp.local_or_column != 0;
}

void LocallyRepairableCode::get_coding_parameters(CodingParameters& cp) const {  // lrc.cpp:14-21
    cp.k = k;
    cp.l = l;
    cp.g = g;
    cp.m = m;
    cp.local_or_column = local_or_column;
}

int LocallyRepairableCode::encode(char** data_ptrs, char** coding_ptrs, int block_size) {  // lrc.cpp:23-30
    std::vector<int> M((size_t)(g + l) * k, 0);
    int rc = make_encoding_matrix(M.data());
    if (rc != ECG_OK) return rc;
    return run_encode(k, g + l, M.data(), data_ptrs, coding_ptrs, block_size);
}

// lrc.cpp:32-42: the LRC local path carries group_id in erasures[failed_num] and overwrites it with -1.
int LocallyRepairableCode::decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures,
                                  int failed_num) {
    if (local_or_column) {
        const int group_id = erasures[failed_num];
        erasures[failed_num] = -1;
        return decode_local(data_ptrs, coding_ptrs, block_size, erasures, failed_num, group_id);
    }
    return decode_global(data_ptrs, coding_ptrs, block_size, erasures, failed_num);
}

int LocallyRepairableCode::decode_global(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures,
                                         int failed_num) {  // lrc.cpp:44-56
    std::vector<int> M((size_t)(g + l) * k, 0);
    int rc = make_encoding_matrix(M.data());
    if (rc != ECG_OK) return rc;
    return run_decode(k, g + l, M.data(), failed_num, erasures, data_ptrs, coding_ptrs, block_size);
}

int LocallyRepairableCode::decode_local(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures,
                                        int failed_num, int group_id) {  // lrc.cpp:58-72
    int min_idx = 0;
    const int gs = get_group_size(group_id, min_idx);
    if (gs < 1) return ECG_EINVAL;
    std::vector<int> gm((size_t)gs, 0);
    int rc = make_group_matrix(gm.data(), group_id, gs);
    if (rc != ECG_OK) return rc;
    return run_decode(gs, 1, gm.data(), failed_num, erasures, data_ptrs, coding_ptrs, block_size);
}

std::vector<int> LocallyRepairableCode::full_matrix() {  // lrc.cpp:107-110
    std::vector<int> f((size_t)(k + g + l) * k, 0);
    get_full_matrix(f.data(), k);
    make_encoding_matrix(&f[(size_t)k * k]);
    return f;
}

std::vector<int> LocallyRepairableCode::group_full_matrix(int gs, int group_id) {  // lrc.cpp:154-156
    std::vector<int> f((size_t)(gs + 1) * gs, 0);
    get_full_matrix(f.data(), gs);
    make_group_matrix(&f[(size_t)gs * gs], group_id, gs);
    return f;
}

int LocallyRepairableCode::remap_local(int idx, int gs, int min_idx) const {  // lrc.cpp:140-152,184-205
    return idx >= k + g ? gs : idx - min_idx;
}

int LocallyRepairableCode::partial_encoding_matrix(std::vector<int> data_idxs, std::vector<int> parity_idxs,
                                                   std::vector<int>& out) {
    if (parity_idxs.empty()) return ECG_EINVAL;
    if (!local_or_column) {  // lrc.cpp:103-113
        if (!ids_in_range(data_idxs, k) || !ids_in_range(parity_idxs, k + g + l)) return ECG_EINVAL;
        std::vector<int> f = full_matrix();
        partial_encoding_matrix_(k, f.data(), data_idxs, parity_idxs, out);
        return ECG_OK;
    }
    // lrc.cpp:128-159 (Opt_Cau_LRC: 1309-1346 through remap_local)
    const int group_id = parity_idxs[0] - k - g;
    int min_idx = -1;
    const int gs = get_group_size(group_id, min_idx);
    if (gs < 1) return ECG_EINVAL;
    for (int& i : data_idxs) i = remap_local(i, gs, min_idx);
    for (int& i : parity_idxs) i = remap_local(i, gs, min_idx);
    if (!ids_in_range(data_idxs, gs) || !ids_in_range(parity_idxs, gs + 1)) return ECG_EINVAL;
    std::vector<int> f = group_full_matrix(gs, group_id);
    partial_encoding_matrix_(gs, f.data(), data_idxs, parity_idxs, out);
    return ECG_OK;
}

int LocallyRepairableCode::partial_decoding_matrix(std::vector<int> lsi, std::vector<int> si, std::vector<int> fi,
                                                   std::vector<int>& out) {
    if (!local_or_column) {  // lrc.cpp:115-126
        if ((int)si.size() > k || !ids_in_range(si, k + g + l) || !ids_in_range(fi, k + g + l)) return ECG_EINVAL;
        std::vector<int> f = full_matrix();
        partial_decoding_matrix_(k, f.data(), lsi, si, fi, out);
        return ECG_OK;
    }
    // lrc.cpp:161-213 (Opt_Cau_LRC: 1348-1413 through remap_local)
    const int gs = (int)si.size();
    int group_id = -1, min_idx = k + g + l;
    for (int idx : si) {
        if (idx >= k + g) group_id = idx - k - g;
        min_idx = std::min(min_idx, idx);
    }
    for (int idx : fi) {
        if (idx >= k + g) group_id = idx - k - g;
        min_idx = std::min(min_idx, idx);
    }
    for (int& i : si) i = remap_local(i, gs, min_idx);
    for (int& i : fi) i = remap_local(i, gs, min_idx);
    for (int& i : lsi) i = remap_local(i, gs, min_idx);
    if (gs < 1 || !ids_in_range(si, gs + 1) || !ids_in_range(fi, gs + 1)) return ECG_EINVAL;
    std::vector<int> f = group_full_matrix(gs, group_id);
    partial_decoding_matrix_(gs, f.data(), lsi, si, fi, out);
    return ECG_OK;
}

int LocallyRepairableCode::check_if_decodable(const std::vector<int>&) { return 1; }  // lrc.h:59

// ---- Azure LRC (lrc.cpp:576-880)
int Azu_LRC::make_encoding_matrix(int* M) {  // lrc.cpp:622-644
    const std::vector<int>& G = cached_vandermonde(k, g);
    if (G.empty()) return ECG_EINVAL;
    std::fill(M, M + (size_t)k * (g + l), 0);
    std::copy(G.begin(), G.end(), M);
    for (int i = 0; i < l; i++)
        for (int j = 0; j < k; j++)
            if (i * r <= j && j < (i + 1) * r) M[(size_t)(i + g) * k + j] = 1;
    return ECG_OK;
}

int Azu_LRC::make_group_matrix(int* gm, int group_id, int size) {  // lrc.cpp:646-656
    if (group_id >= 0 && group_id < l) {
        const int gs = std::min(r, k - group_id * r);
        for (int j = 0; j < gs && j < size; j++) gm[j] = 1;
    }
    return ECG_OK;
}

int Azu_LRC::bid2gid(int b) {  // lrc.cpp:665-676
    if (b < k) return b / r;
    if (b < k + g) return l;
    return b - k - g;
}

int Azu_LRC::idxingroup(int b) {  // lrc.cpp:678-691
    if (b < k) return b % r;
    if (b < k + g) return b - k;
    if (b - k - g < l - 1) return r;
    return k % r == 0 ? r : k % r;
}

int Azu_LRC::get_group_size(int group_id, int& min_idx) {  // lrc.cpp:693-704
    min_idx = group_id * r;
    if (group_id < l - 1) return r;
    if (group_id == l - 1) return k % r == 0 ? r : k % r;
    min_idx = k;
    return g;
}

int Azu_LRC::check_if_decodable(const std::vector<int>& failure_idxs) {  // lrc.cpp:576-620
    std::vector<int> b2g(k, 0), fd(l, 0), slp(l, 1);
    int sgp = g, idx = 0;
    for (int i = 0; i < l; i++) {
        const int gs = std::min(r, k - i * r);
        for (int j = 0; j < gs; j++) b2g[idx++] = i;
    }
    for (int b : failure_idxs) {
        if (b < k) fd[b2g[b]] += 1;
        else if (b < k + g) sgp -= 1;
        else slp[b - k - g] -= 1;
    }
    for (int i = 0; i < l; i++)
        if (slp[i] && slp[i] <= fd[i]) {
            fd[i] -= slp[i];
            slp[i] = 0;
        }
    for (int i = 0; i < l; i++) {
        if (sgp >= fd[i]) {
            sgp -= fd[i];
            fd[i] = 0;
        } else {
            return 0;
        }
    }
    return 1;
}

std::string Azu_LRC::self_information() const {
    return "Azure_LRC(" + std::to_string(k) + "," + std::to_string(l) + "," + std::to_string(g) + ")";
}

// L (l x (k+g)) * [I_k ; G] -> local rows (Azure+1 lrc.cpp:951-974, Optimal lrc.cpp:1183-1209)
static std::vector<int> mix_local(const std::vector<int>& L, const std::vector<int>& G, int k, int g, int l) {
    std::vector<int> dg((size_t)(k + g) * k, 0);
    for (int i = 0; i < k; i++) dg[(size_t)i * k + i] = 1;
    std::copy(G.begin(), G.end(), dg.begin() + (size_t)k * k);
    return matrix_multiply(L.data(), dg.data(), l, k + g, k + g, k);
}

// ---- Azure LRC + 1 (lrc.cpp:881-1094)
int Azu_LRC_1::make_encoding_matrix(int* M) {  // lrc.cpp:933-981
    const std::vector<int>& G = cached_vandermonde(k, g);
    if (G.empty() || l < 1) return ECG_EINVAL;
    std::fill(M, M + (size_t)k * (g + l), 0);
    std::copy(G.begin(), G.end(), M);
    std::vector<int> L((size_t)l * (k + g), 0);
    int idx = 0;
    for (int i = 0; i < l - 1; i++)
        for (int j = 0; j < std::min(r, k - i * r); j++) L[(size_t)i * (k + g) + idx++] = 1;
    for (int j = 0; j < g; j++) L[(size_t)(l - 1) * (k + g) + idx++] = 1;
    std::vector<int> mix = mix_local(L, G, k, g, l);
    std::copy(mix.begin(), mix.end(), M + (size_t)g * k);
    return ECG_OK;
}

int Azu_LRC_1::make_group_matrix(int* gm, int group_id, int size) {  // lrc.cpp:983-999
    if (group_id == l - 1) {
        for (int j = 0; j < g && j < size; j++) gm[j] = 1;
        return ECG_OK;
    }
    if (group_id >= 0 && group_id < l - 1) {
        const int gs = std::min(r, k - group_id * r);
        for (int j = 0; j < gs && j < size; j++) gm[j] = 1;
    }
    return ECG_OK;
}

int Azu_LRC_1::bid2gid(int b) {  // lrc.cpp:1008-1019
    if (b < k) return b / r;
    if (b < k + g) return l - 1;
    return b - k - g;
}

int Azu_LRC_1::idxingroup(int b) {  // lrc.cpp:1021-1036
    if (b < k) return b % r;
    if (b < k + g) return b - k;
    if (b - k - g < l - 2) return r;
    if (b - k - g == l - 2) return k % r == 0 ? r : k % r;
    return g;
}

int Azu_LRC_1::get_group_size(int group_id, int& min_idx) {  // lrc.cpp:1038-1049
    min_idx = group_id * r;
    if (group_id < l - 2) return r;
    if (group_id == l - 2) return k % r == 0 ? r : k % r;
    min_idx = k;
    return g;
}

std::string Azu_LRC_1::self_information() const {
    return "Azure_LRC+1(" + std::to_string(k) + "," + std::to_string(l) + "," + std::to_string(g) + ")";
}

// ---- Optimal LRC (lrc.cpp:1096-1307)
int Opt_LRC::make_encoding_matrix(int* M) {  // lrc.cpp:1168-1215
    const std::vector<int>& G = cached_vandermonde(k, g);
    if (G.empty()) return ECG_EINVAL;
    std::fill(M, M + (size_t)k * (g + l), 0);
    std::copy(G.begin(), G.end(), M);
    std::vector<int> L((size_t)l * (k + g), 0);
    int idx = 0;
    for (int i = 0; i < l; i++)
        for (int j = 0; j < std::min(r, k + g - i * r); j++) L[(size_t)i * (k + g) + idx++] = 1;
    std::vector<int> mix = mix_local(L, G, k, g, l);
    std::copy(mix.begin(), mix.end(), M + (size_t)g * k);
    return ECG_OK;
}

int Opt_LRC::make_group_matrix(int* gm, int group_id, int size) {  // lrc.cpp:1217-1227
    if (group_id >= 0 && group_id < l) {
        const int gs = std::min(r, k + g - group_id * r);
        for (int j = 0; j < gs && j < size; j++) gm[j] = 1;
    }
    return ECG_OK;
}

int Opt_LRC::bid2gid(int b) { return b < k + g ? b / r : b - k - g; }  // lrc.cpp:1236-1245

int Opt_LRC::idxingroup(int b) {  // lrc.cpp:1247-1258
    if (b < k + g) return b % r;
    if (b - k - g < l - 1) return r;
    return (k + g) % r == 0 ? r : (k + g) % r;
}

int Opt_LRC::get_group_size(int group_id, int& min_idx) {  // lrc.cpp:1260-1268
    min_idx = group_id * r;
    if (group_id < l - 1) return r;
    return (k + g) % r == 0 ? r : (k + g) % r;
}

std::string Opt_LRC::self_information() const {
    return "Optimal_LRC(" + std::to_string(k) + "," + std::to_string(l) + "," + std::to_string(g) + ")";
}

// ---- Optimal Cauchy LRC (lrc.cpp:1309-1755)
int Opt_Cau_LRC::make_encoding_matrix(int* M) {  // lrc.cpp:1485-1518
    const std::vector<int>& C = cached_cauchy_good(k, g + 1);
    if (C.empty()) return g + 1 == 2 ? ECG_EUNPINNED : ECG_EINVAL;
    std::fill(M, M + (size_t)k * (g + l), 0);
    std::copy(C.begin(), C.begin() + (size_t)g * k, M);
    int d = 0;
    for (int i = 0; i < l; i++)
        for (int j = 0; j < k; j++)
            if (i * r <= j && j < (i + 1) * r) M[(size_t)(i + g) * k + j] = C[(size_t)g * k + d++];
    for (int i = 0; i < l; i++)  // galois_region_xor of every global row into every local row
        for (int j = 0; j < g; j++)
            for (int t = 0; t < k; t++) M[(size_t)(i + g) * k + t] ^= C[(size_t)j * k + t];
    return ECG_OK;
}

int Opt_Cau_LRC::make_group_matrix(int* gm, int group_id, int size) {  // lrc.cpp:1574-1591
    const std::vector<int>& C = cached_cauchy_good(k, g + 1);
    if (C.empty()) return g + 1 == 2 ? ECG_EUNPINNED : ECG_EINVAL;
    int idx = 0;
    for (int i = 0; i < l; i++) {
        const int gs = std::min(r, k - i * r);
        for (int j = 0; j < gs; j++) {
            if (i == group_id && j < size) gm[j] = C[(size_t)g * k + idx];
            idx++;
        }
        for (int j = gs; j < gs + g; j++)
            if (i == group_id && j < size) gm[j] = 1;
    }
    return ECG_OK;
}

int Opt_Cau_LRC::bid2gid(int b) {  // lrc.cpp:1600-1611
    if (b < k) return b / r;
    if (b < k + g) return l;
    return b - k - g;
}

int Opt_Cau_LRC::idxingroup(int b) {  // lrc.cpp:1613-1626
    if (b < k) return b % r;
    if (b < k + g) return b - k + r;
    if (b - k - g < l - 1) return r + g;
    return k % r == 0 ? r + g : k % r + g;
}

int Opt_Cau_LRC::get_group_size(int group_id, int& min_idx) {  // lrc.cpp:1628-1639
    min_idx = group_id * r;
    if (group_id < l - 1) return r + g;
    if (group_id == l - 1) return (k % r == 0 ? r : k % r) + g;
    min_idx = k;
    return g;
}

int Opt_Cau_LRC::remap_local(int idx, int gs, int min_idx) const {  // lrc.cpp:1320-1340
    if (idx >= k + g) return gs;
    if (idx >= k) return gs - g + idx - k;
    return idx - min_idx;
}

std::string Opt_Cau_LRC::self_information() const {
    return "Optimal_Cauchy_LRC(" + std::to_string(k) + "," + std::to_string(l) + "," + std::to_string(g) + ")";
}

// ---- Uniform Cauchy LRC (lrc.cpp:2025-2310)
int Uni_Cau_LRC::make_encoding_matrix(int* M) {  // lrc.cpp:2097-2156
    const std::vector<int>& C = cached_cauchy_good(k, g + 1);
    if (C.empty()) return g + 1 == 2 ? ECG_EUNPINNED : ECG_EINVAL;
    std::fill(M, M + (size_t)k * (g + l), 0);
    std::copy(C.begin(), C.begin() + (size_t)g * k, M);
    std::vector<int> L((size_t)l * k, 0);
    int d = 0, l_idx = 0;
    for (int i = 0; i < l && d < k; i++) {
        const int gs = std::min(r, k + g - i * r);
        for (int j = 0; j < gs && d < k; j++, d++) L[(size_t)i * k + d] = C[(size_t)g * k + d];
        l_idx = i;
    }
    int g_idx = 0;
    for (int i = l_idx; i < l; i++) {
        const int gs = std::min(r, k + g - i * r);
        const int sub = gs < r ? g - g_idx : (i + 1) * r - (k + g_idx);
        for (int j = 0; j < sub && g_idx < g; j++, g_idx++)
            for (int t = 0; t < k; t++) L[(size_t)i * k + t] ^= C[(size_t)g_idx * k + t];
    }
    std::copy(L.begin(), L.end(), M + (size_t)g * k);
    return ECG_OK;
}

int Uni_Cau_LRC::make_group_matrix(int* gm, int group_id, int size) {  // lrc.cpp:2213-2230
    const std::vector<int>& C = cached_cauchy_good(k, g + 1);
    if (C.empty()) return g + 1 == 2 ? ECG_EUNPINNED : ECG_EINVAL;
    int idx = 0;
    for (int i = 0; i < l; i++) {
        const int gs = std::min(r, k + g - i * r);
        for (int j = 0; j < gs; j++) {
            if (i == group_id && j < size) gm[j] = idx < k ? C[(size_t)g * k + idx] : 1;
            idx++;
        }
    }
    return ECG_OK;
}

int Uni_Cau_LRC::bid2gid(int b) { return b < k + g ? b / r : b - k - g; }  // lrc.cpp:2239-2248

int Uni_Cau_LRC::idxingroup(int b) {  // lrc.cpp:2250-2261
    if (b < k + g) return b % r;
    if (b - k - g < l - 1) return r;
    return (k + g) % r == 0 ? r : (k + g) % r;
}

int Uni_Cau_LRC::get_group_size(int group_id, int& min_idx) {  // lrc.cpp:2263-2271
    min_idx = group_id * r;
    if (group_id < l - 1) return r;
    return (k + g) % r == 0 ? r : (k + g) % r;
}

std::string Uni_Cau_LRC::self_information() const {
    return "Uniform_Cauchy_LRC(" + std::to_string(k) + "," + std::to_string(l) + "," + std::to_string(g) + ")";
}

// ================================================================================== Product codes

void ProductCode::init_coding_parameters(const CodingParameters& cp) {  // pc.cpp:5-18
    k1 = cp.k1;
    m1 = cp.m1;
    k2 = cp.k2;
    m2 = cp.m2;
    k = k1 * k2;
    m = (k1 + m1) * (k2 + m2) - k;
    row_code.k = k1;
    row_code.m = m1;
    col_code.k = k2;
    col_code.m = m2;
    local_or_column = cp.local_or_column != 0;
}

void ProductCode::get_coding_parameters(CodingParameters& cp) const {  // pc.cpp:20-29
    cp.k1 = k1;
    cp.m1 = m1;
    cp.k2 = k2;
    cp.m2 = m2;
    cp.k = k;
    cp.m = m;
    cp.local_or_column = local_or_column;
}

// [row][col] -> id in the data (k) ++ coding (m) block space; pc.cpp:31-38, 86-108 ordering
std::vector<std::vector<int>> ProductCode::block_map() const {
    std::vector<std::vector<int>> bm(k2 + m2, std::vector<int>(k1 + m1, -1));
    int di = 0, pi = 0;
    for (int i = 0; i < k2; i++)
        for (int j = 0; j < k1 + m1; j++) bm[i][j] = j < k1 ? di++ : k + pi++;
    int gi = k2 * m1 + m2 * k1;
    for (int i = k2; i < k2 + m2; i++)
        for (int j = 0; j < k1 + m1; j++) {
            if (j < k1) bm[i][j] = k + pi++;
            else if (has_global()) bm[i][j] = k + gi++;
        }
    return bm;
}

// The row codes, then the column codes over the data and the row parities (pc.cpp:39-76), planned as one call
// and composed (finish_plan): each data block is read once, the row parities are not re-read.
int ProductCode::encode(char** data_ptrs, char** coding_ptrs, int block_size) {
    thread_local std::vector<int> key;
    key.assign({4});
    state_key(key);
    const CallPlan* cp = nullptr;
    const int rc = run_planned(key, [&](Plan& p) {
        for (int i = 0; i < k2; i++) {
            std::vector<int> d(k1), c(m1);
            for (int j = 0; j < k1; j++) d[j] = i * k1 + j;
            for (int j = 0; j < m1; j++) c[j] = k + i * m1 + j;
            if (int r = rowc().plan_encode(p, d, c); r != ECG_OK) return r;
        }
        for (int i = 0; i < k1 + m1; i++) {
            std::vector<int> d(k2), c(m2);
            for (int j = 0; j < k2; j++) d[j] = i < k1 ? j * k1 + i : k + j * m1 + i - k1;
            for (int j = 0; j < m2; j++)
                c[j] = i < k1 ? k + k2 * m1 + j * k1 + i : k + k2 * m1 + k1 * m2 + j * m1 + i - k1;
            if (int r = colc().plan_encode(p, d, c); r != ECG_OK) return r;
        }
        return (int)ECG_OK;
    }, cp);
    if (rc != ECG_OK) return rc;
    return run(cp->ops, data_ptrs, k, coding_ptrs, m, block_size);
}

// Iterative control flow of pc.cpp:79-195 (and HVPC pc.cpp:921-1029 with ncols = k1, nrows = k2).
int ProductCode::plan_iterative_decode(Plan& p, int* erasures, int failed_num, int ncols, int nrows) {
    const std::vector<std::vector<int>> bm = block_map();
    std::vector<std::vector<int>> fmap(k2 + m2, std::vector<int>(k1 + m1, 0));
    std::vector<int> frc(k2 + m2, 0), fcc(k1 + m1, 0);
    for (int i = 0; i < failed_num; i++) {
        int r = -1, c = -1;
        bid2rowcol(erasures[i], r, c);
        if (r < 0 || r >= k2 + m2 || c < 0 || c >= k1 + m1) return ECG_EINVAL;
        fmap[r][c] = 1;
        frc[r]++;
        fcc[c]++;
    }
    while (failed_num > 0) {
        for (int i = 0; i < ncols; i++) {
            if (fcc[i] > 0 && fcc[i] <= m2) {
                std::vector<int> er, d(k2), c(m2);
                for (int jj = 0; jj < k2; jj++) {
                    if (fmap[jj][i]) er.push_back(jj);
                    d[jj] = bm[jj][i];
                }
                for (int jj = 0; jj < m2; jj++) {
                    if (fmap[jj + k2][i]) er.push_back(jj + k2);
                    c[jj] = bm[jj + k2][i];
                }
                er.push_back(-1);
                (void)colc().plan_decode(p, d, c, er.data(), fcc[i]);  // failure: "[Decode] Failed!", continue
                for (int jj = 0; jj < k2 + m2; jj++)
                    if (fmap[jj][i]) {
                        fmap[jj][i] = 0;
                        failed_num--;
                        frc[jj]--;
                        fcc[i]--;
                    }
            }
        }
        if (failed_num == 0) break;
        int max_row = -1;
        for (int i = 0; i < nrows; i++) {
            if (frc[i] > 0 && frc[i] <= m1) {
                max_row = i;
                std::vector<int> er, d(k1), c(m1);
                for (int jj = 0; jj < k1; jj++) {
                    if (fmap[i][jj]) er.push_back(jj);
                    d[jj] = bm[i][jj];
                }
                for (int jj = 0; jj < m1; jj++) {
                    if (fmap[i][jj + k1]) er.push_back(jj + k1);
                    c[jj] = bm[i][jj + k1];
                }
                er.push_back(-1);
                (void)rowc().plan_decode(p, d, c, er.data(), frc[i]);
                for (int jj = 0; jj < k1 + m1; jj++)
                    if (fmap[i][jj]) {
                        fmap[i][jj] = 0;
                        failed_num--;
                        frc[i]--;
                        fcc[jj]--;
                    }
            }
        }
        if (max_row == -1) return ECG_EUNDECODABLE;  // "Undecodable!!" (work planned so far still runs)
    }
    return ECG_OK;
}

// Iterative decode (pc.cpp:79-195) planned on the host, composed into one pass where it can be (finish_plan).
int ProductCode::decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) {
    return decode_iterative(data_ptrs, coding_ptrs, block_size, erasures, failed_num, k1 + m1, k2 + m2);
}

int ProductCode::decode_iterative(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num,
                                  int ncols, int nrows) {
    const int nf = std::max(0, failed_num);
    thread_local std::vector<int> key;
    key.assign({5, ncols, nrows, failed_num});
    state_key(key);
    key.insert(key.end(), erasures, erasures + nf);
    const CallPlan* cp = nullptr;
    const int status = run_planned(key, [&](Plan& p) {
        std::vector<int> er(erasures, erasures + nf);  // the planner reads the list only
        er.push_back(-1);
        return plan_iterative_decode(p, er.data(), failed_num, ncols, nrows);
    }, cp);
    if (!cp) return status;
    const int rc = run(cp->ops, data_ptrs, k, coding_ptrs, m, block_size);
    return rc != ECG_OK ? rc : status;
}

int ProductCode::check_if_decodable(const std::vector<int>& failure_idxs) {  // pc.cpp:198-255
    int failed_num = (int)failure_idxs.size();
    std::vector<std::vector<int>> fmap(k2 + m2, std::vector<int>(k1 + m1, 0));
    std::vector<int> frc(k2 + m2, 0), fcc(k1 + m1, 0);
    for (int b : failure_idxs) {
        int r, c;
        bid2rowcol(b, r, c);
        if (r < 0 || r >= k2 + m2 || c < 0 || c >= k1 + m1) return ECG_EINVAL;
        fmap[r][c] = 1;
        frc[r]++;
        fcc[c]++;
    }
    const int ncols = has_global() ? k1 + m1 : k1, nrows = has_global() ? k2 + m2 : k2;
    while (failed_num > 0) {
        for (int i = 0; i < ncols; i++)
            if (fcc[i] > 0 && fcc[i] <= m2)
                for (int jj = 0; jj < k2 + m2; jj++)
                    if (fmap[jj][i]) {
                        fmap[jj][i] = 0;
                        failed_num--;
                        frc[jj]--;
                        fcc[i]--;
                    }
        if (failed_num == 0) break;
        int max_row = -1;
        for (int i = 0; i < nrows; i++)
            if (frc[i] > 0 && frc[i] <= m1) {
                max_row = i;
                for (int jj = 0; jj < k1 + m1; jj++)
                    if (fmap[i][jj]) {
                        fmap[i][jj] = 0;
                        failed_num--;
                        frc[i]--;
                        fcc[jj]--;
                    }
            }
        if (max_row == -1) return 0;
    }
    return 1;
}

int ProductCode::partial_encoding_matrix(std::vector<int> data_idxs, std::vector<int> parity_idxs,
                                         std::vector<int>& out) {  // pc.cpp:257-288
    int r, c;
    for (int& i : data_idxs) {
        bid2rowcol(i, r, c);
        i = local_or_column ? r : c;
    }
    for (int& i : parity_idxs) {
        bid2rowcol(i, r, c);
        i = local_or_column ? r : c;
    }
    RSCode& code = local_or_column ? partial_col() : partial_row();
    return code.partial_encoding_matrix(data_idxs, parity_idxs, out);
}

int ProductCode::partial_decoding_matrix(std::vector<int> lsi, std::vector<int> si, std::vector<int> fi,
                                         std::vector<int>& out) {  // pc.cpp:290-324
    int r, c;
    for (std::vector<int>* v : {&lsi, &si, &fi})
        for (int& i : *v) {
            bid2rowcol(i, r, c);
            i = local_or_column ? r : c;
        }
    RSCode& code = local_or_column ? partial_col() : partial_row();
    return code.partial_decoding_matrix(lsi, si, fi, out);
}

int ProductCode::rowcol2bid(int row, int col) const {  // pc.cpp:326-340
    if (row < k2 && col < k1) return row * k1 + col;
    if (row < k2) return k1 * k2 + row * m1 + (col - k1);
    if (col < k1) return (k1 + m1) * k2 + (row - k2) * k1 + col;
    return (k1 + m1) * k2 + k1 * m2 + (row - k2) * m1 + (col - k1);
}

void ProductCode::bid2rowcol(int bid, int& row, int& col) const {  // pc.cpp:342-359
    if (bid < k1 * k2) {
        row = bid / k1;
        col = bid % k1;
    } else if (bid < (k1 + m1) * k2) {
        const int t = bid - k1 * k2;
        row = t / m1;
        col = t % m1 + k1;
    } else if (bid < (k1 + m1) * k2 + k1 * m2) {
        const int t = bid - (k1 + m1) * k2;
        row = t / k1 + k2;
        col = t % k1;
    } else {
        const int t = bid - (k1 + m1) * k2 - k1 * m2;
        row = t / m1 + k2;
        col = t % m1 + k1;
    }
}

int ProductCode::oldbid2newbid_for_merge(int old_block_id, int x, int seri_num, bool vertical) {  // pc.cpp:361-376
    int row = -1, col = -1;
    bid2rowcol(old_block_id, row, col);
    if (vertical) {
        row += seri_num * k2;
        ProductCode pc(k1, m1, x * k2, m2);
        return pc.rowcol2bid(row, col);
    }
    col += seri_num * k1;
    ProductCode pc(x * k1, m1, k2, m2);
    return pc.rowcol2bid(row, col);
}

std::string ProductCode::self_information() const {
    return "PC(" + std::to_string(k1) + "," + std::to_string(m1) + "," + std::to_string(k2) + "," +
           std::to_string(m2) + ")";
}

void HPC::init_coding_parameters(const CodingParameters& cp) {  // pc.cpp:553-574
    ProductCode::init_coding_parameters(cp);
    e_row_code.k = cp.k1;
    e_row_code.m = cp.m1;
    e_row_code.x = cp.x;
    e_row_code.seri_num = cp.seri_num;
    e_col_code.k = cp.k2;
    e_col_code.m = cp.m2;
    e_col_code.x = cp.x;
    e_col_code.seri_num = cp.seri_num;
}

int HPC::oldbid2newbid_for_merge(int old_block_id, int, int, bool vertical) {  // pc.cpp:838-856
    int row = -1, col = -1;
    bid2rowcol(old_block_id, row, col);
    if (vertical) {
        row += e_col_code.seri_num * k2;
        ProductCode pc(k1, m1, e_col_code.x * k2, m2);
        return pc.rowcol2bid(row, col);
    }
    col += e_row_code.seri_num * k1;
    ProductCode pc(e_row_code.x * k1, m1, k2, m2);
    return pc.rowcol2bid(row, col);
}

std::string HPC::self_information() const {
    return "HPC(" + std::to_string(k1) + "," + std::to_string(m1) + "," + std::to_string(k2) + "," +
           std::to_string(m2) + "|" + std::to_string(e_col_code.x) + "," + std::to_string(e_col_code.seri_num) + ")";
}

void HVPC::init_coding_parameters(const CodingParameters& cp) {  // pc.cpp:869-882
    ProductCode::init_coding_parameters(cp);
    m = k1 * m2 + k2 * m1;
}

int HVPC::encode(char** data_ptrs, char** coding_ptrs, int block_size) {  // pc.cpp:890-918
    thread_local std::vector<int> key;
    key.assign({4});
    state_key(key);
    const CallPlan* cp = nullptr;
    const int rc = run_planned(key, [&](Plan& p) {
        for (int i = 0; i < k2; i++) {
            std::vector<int> d(k1), c(m1);
            for (int j = 0; j < k1; j++) d[j] = i * k1 + j;
            for (int j = 0; j < m1; j++) c[j] = k + i * m1 + j;
            if (int r = row_code.plan_encode(p, d, c); r != ECG_OK) return r;
        }
        for (int i = 0; i < k1; i++) {
            std::vector<int> d(k2), c(m2);
            for (int j = 0; j < k2; j++) d[j] = j * k1 + i;
            for (int j = 0; j < m2; j++) c[j] = k + k2 * m1 + j * k1 + i;
            if (int r = col_code.plan_encode(p, d, c); r != ECG_OK) return r;
        }
        return (int)ECG_OK;
    }, cp);
    if (rc != ECG_OK) return rc;
    return run(cp->ops, data_ptrs, k, coding_ptrs, m, block_size);
}

// pc.cpp:921-1029: the iterative decode over the k1 data columns and k2 data rows only
int HVPC::decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) {
    return decode_iterative(data_ptrs, coding_ptrs, block_size, erasures, failed_num, k1, k2);
}

int HVPC::check_if_decodable(const std::vector<int>& f) { return ProductCode::check_if_decodable(f); }

std::string HVPC::self_information() const {
    return "HVPC(" + std::to_string(k1) + "," + std::to_string(m1) + "," + std::to_string(k2) + "," +
           std::to_string(m2) + ")";
}

// ================================================================================== factory

ErasureCode* ec_factory(int ec_type, const CodingParameters& cp) {  // metadata.cpp:48-77
    switch (ec_type) {
        case ECG_RS: return new RSCode(cp.k, cp.m);
        case ECG_ERS: {
            auto* ec = new EnlargedRSCode(cp.k, cp.m);
            ec->init_coding_parameters(cp);
            return ec;
        }
        case ECG_AZURE_LRC: return cp.l > 0 ? new Azu_LRC(cp.k, cp.l, cp.g) : nullptr;
        case ECG_AZURE_LRC_1: return cp.l > 1 ? new Azu_LRC_1(cp.k, cp.l, cp.g) : nullptr;
        case ECG_OPTIMAL_LRC: return cp.l > 0 ? new Opt_LRC(cp.k, cp.l, cp.g) : nullptr;
        case ECG_OPTIMAL_CAUCHY_LRC: return cp.l > 0 ? new Opt_Cau_LRC(cp.k, cp.l, cp.g) : nullptr;
        case ECG_UNIFORM_CAUCHY_LRC: return cp.l > 0 ? new Uni_Cau_LRC(cp.k, cp.l, cp.g) : nullptr;
        case ECG_PC: return new ProductCode(cp.k1, cp.m1, cp.k2, cp.m2);
        case ECG_HIERACHICAL_PC: {
            auto* ec = new HPC(cp.k1, cp.m1, cp.k2, cp.m2);
            ec->init_coding_parameters(cp);
            return ec;
        }
        case ECG_HV_PC: return new HVPC(cp.k1, cp.m1, cp.k2, cp.m2);
        default: return nullptr;
    }
}

}  // namespace ecg
