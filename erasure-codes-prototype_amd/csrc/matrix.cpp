// Host-side matrix construction and decode planning.  See matrix.hpp.
#include "matrix.hpp"

#include <unordered_map>

#include <algorithm>

#include <map>
#include <mutex>

#include "gf256.hpp"

namespace ecg {

// ------------------------------------------------------------------------------------------------
// Vandermonde (Jerasure reed_sol.c semantics, w = 8)

namespace {

std::vector<int> extended_vandermonde(int rows, int cols) {
    std::vector<int> v((size_t)rows * cols, 0);
    v[0] = 1;
    if (rows == 1) return v;
    v[(size_t)(rows - 1) * cols + (cols - 1)] = 1;
    if (rows == 2) return v;
    for (int i = 1; i < rows - 1; i++) {
        int p = 1;
        for (int j = 0; j < cols; j++) {
            v[(size_t)i * cols + j] = p;
            p = gf::mul(p, i);
        }
    }
    return v;
}

// Column-reduce the extended Vandermonde matrix to [I; X], then normalise row `cols` and column 0
// of the remaining rows to ones.
std::vector<int> big_vandermonde_distribution(int rows, int cols) {
    if (cols >= rows || rows > 256) return {};
    std::vector<int> d = extended_vandermonde(rows, cols);
    auto at = [&](int r, int c) -> int& { return d[(size_t)r * cols + c]; };
    for (int i = 1; i < cols; i++) {
        int r = i;
        while (r < rows && at(r, i) == 0) r++;
        if (r == rows) return {};
        if (r != i)
            for (int c = 0; c < cols; c++) std::swap(at(r, c), at(i, c));
        if (at(i, i) != 1) {
            const int s = gf::div(1, at(i, i));
            for (int rr = 0; rr < rows; rr++) at(rr, i) = gf::mul(s, at(rr, i));
        }
        for (int j = 0; j < cols; j++) {
            const int e = at(i, j);
            if (j == i || e == 0) continue;
            for (int rr = 0; rr < rows; rr++) at(rr, j) ^= gf::mul(e, at(rr, i));
        }
    }
    for (int j = 0; j < cols; j++) {
        const int e = at(cols, j);
        if (e == 1) continue;
        const int s = gf::div(1, e);
        for (int rr = cols; rr < rows; rr++) at(rr, j) = gf::mul(s, at(rr, j));
    }
    for (int rr = cols + 1; rr < rows; rr++) {
        const int e = at(rr, 0);
        if (e == 1) continue;
        const int s = gf::div(1, e);
        for (int j = 0; j < cols; j++) at(rr, j) = gf::mul(at(rr, j), s);
    }
    return d;
}

}  // namespace

std::vector<int> reed_sol_vandermonde_coding_matrix(int k, int m) {
    if (k < 1 || m < 1) return {};
    std::vector<int> d = big_vandermonde_distribution(k + m, k);
    if (d.empty()) return {};
    return std::vector<int>(d.begin() + (size_t)k * k, d.end());
}

// ------------------------------------------------------------------------------------------------
// Cauchy (Jerasure cauchy.c semantics, w = 8)

int cauchy_n_ones(int e) {
    int total = 0;
    int x = e & 0xff;
    for (int i = 0; i < 8; i++) {
        total += __builtin_popcount((unsigned)x);
        x = gf::mul(x, 2);
    }
    return total;
}

std::vector<int> cauchy_original_coding_matrix(int k, int m) {
    if (k < 1 || m < 1 || k + m > 256) return {};
    std::vector<int> M((size_t)k * m);
    for (int i = 0; i < m; i++)
        for (int j = 0; j < k; j++) M[(size_t)i * k + j] = gf::div(1, i ^ (m + j));
    return M;
}

void cauchy_improve_coding_matrix(int k, int m, std::vector<int>& M) {
    for (int j = 0; j < k; j++) {
        if (M[j] == 1) continue;
        const int s = gf::div(1, M[j]);
        for (int i = 0; i < m; i++) M[(size_t)i * k + j] = gf::mul(M[(size_t)i * k + j], s);
    }
    for (int i = 1; i < m; i++) {
        int* row = &M[(size_t)i * k];
        int best = 0;
        for (int j = 0; j < k; j++) best += cauchy_n_ones(row[j]);
        int best_j = -1;
        for (int j = 0; j < k; j++) {
            if (row[j] == 1) continue;
            const int s = gf::div(1, row[j]);
            int ones = 0;
            for (int x = 0; x < k; x++) ones += cauchy_n_ones(gf::mul(row[x], s));
            if (ones < best) {
                best = ones;
                best_j = j;
            }
        }
        if (best_j >= 0) {
            const int s = gf::div(1, row[best_j]);
            for (int j = 0; j < k; j++) row[j] = gf::mul(row[j], s);
        }
    }
}

namespace {
std::mutex g_builder_mu;
std::map<std::pair<int, int>, std::vector<int>> g_vand, g_cauchy;
}  // namespace

const std::vector<int>& cached_vandermonde(int k, int m) {
    std::lock_guard<std::mutex> lk(g_builder_mu);
    auto it = g_vand.find({k, m});
    if (it == g_vand.end()) it = g_vand.emplace(std::make_pair(k, m), reed_sol_vandermonde_coding_matrix(k, m)).first;
    return it->second;
}

const std::vector<int>& cached_cauchy_good(int k, int m) {
    std::lock_guard<std::mutex> lk(g_builder_mu);
    auto it = g_cauchy.find({k, m});
    if (it == g_cauchy.end()) it = g_cauchy.emplace(std::make_pair(k, m), cauchy_good_general_coding_matrix(k, m)).first;
    return it->second;
}

std::vector<int> cauchy_good_general_coding_matrix(int k, int m) {
    if (m == 2 && k <= 255) return {};  // Jerasure cbest_8 table: unpinned offline
    std::vector<int> M = cauchy_original_coding_matrix(k, m);
    if (M.empty()) return {};
    cauchy_improve_coding_matrix(k, m, M);
    return M;
}

// ------------------------------------------------------------------------------------------------
// Matrix algebra (Jerasure jerasure.c semantics)

int invert_matrix(std::vector<int>& mat, std::vector<int>& inv, int rows) {
    const int n = rows;
    inv.assign((size_t)n * n, 0);
    for (int i = 0; i < n; i++) inv[(size_t)i * n + i] = 1;
    auto A = [&](int r, int c) -> int& { return mat[(size_t)r * n + c]; };
    auto V = [&](int r, int c) -> int& { return inv[(size_t)r * n + c]; };
    for (int i = 0; i < n; i++) {
        if (A(i, i) == 0) {
            int j = i + 1;
            while (j < n && A(j, i) == 0) j++;
            if (j == n) return -1;
            for (int c = 0; c < n; c++) {
                std::swap(A(i, c), A(j, c));
                std::swap(V(i, c), V(j, c));
            }
        }
        if (A(i, i) != 1) {
            const int s = gf::div(1, A(i, i));
            for (int c = 0; c < n; c++) {
                A(i, c) = gf::mul(A(i, c), s);
                V(i, c) = gf::mul(V(i, c), s);
            }
        }
        for (int j = i + 1; j < n; j++) {
            const int e = A(j, i);
            if (e == 0) continue;
            for (int c = 0; c < n; c++) {
                A(j, c) ^= gf::mul(e, A(i, c));
                V(j, c) ^= gf::mul(e, V(i, c));
            }
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        for (int j = 0; j < i; j++) {
            const int e = A(j, i);
            if (e == 0) continue;
            A(j, i) = 0;
            for (int c = 0; c < n; c++) V(j, c) ^= gf::mul(e, V(i, c));
        }
    }
    return 0;
}

std::vector<int> matrix_multiply(const int* m1, const int* m2, int r1, int c1, int r2, int c2) {
    std::vector<int> p((size_t)r1 * c2, 0);
    for (int i = 0; i < r1; i++)
        for (int j = 0; j < c2; j++) {
            int acc = 0;
            for (int t = 0; t < r2; t++) acc ^= gf::mul(m1[(size_t)i * c1 + t], m2[(size_t)t * c2 + j]);
            p[(size_t)i * c2 + j] = acc;
        }
    return p;
}

// ------------------------------------------------------------------------------------------------
// Planning

bool op_is_binary(const LinearOp& op) {
    for (uint8_t c : op.coef)
        if (c > 1) return false;
    return true;
}

LinearOp plan_matrix_encode(int k, int m, const int* matrix) {
    LinearOp op;
    op.src_ids.reserve(k);
    op.dst_ids.reserve(m);
    op.coef.reserve((size_t)k * m);
    for (int j = 0; j < k; j++) op.src_ids.push_back(j);
    for (int i = 0; i < m; i++) {
        const int* row = matrix + (size_t)i * k;
        bool any = false;
        for (int j = 0; j < k; j++) any |= (row[j] & 0xff) != 0;
        if (!any) continue;
        op.dst_ids.push_back(k + i);
        for (int j = 0; j < k; j++) op.coef.push_back((uint8_t)(row[j] & 0xff));
    }
    return op;
}

namespace {

// Symbolic replay: content[b] = linear combination of the ORIGINAL block contents.
struct Replay {
    int n;
    std::vector<std::vector<uint8_t>> content;
    std::vector<int> written;       // in first-write order
    std::vector<LinearOp> steps;    // one op per executed dot product (fallback plan)

    explicit Replay(int n_) : n(n_), content(n_, std::vector<uint8_t>(n_, 0)) {
        for (int b = 0; b < n; b++) content[b][b] = 1;
    }

    // jerasure_matrix_dotprod(k, w, row, src_ids, dest): an all-zero row writes nothing.
    void dotprod(int k, const int* row, const int* src_ids, int dest) {
        std::vector<uint8_t> acc(n, 0);
        LinearOp step;
        bool any = false;
        for (int i = 0; i < k; i++) {
            const int c = row[i] & 0xff;
            if (c == 0) continue;
            any = true;
            const int src = src_ids ? src_ids[i] : i;
            for (int b = 0; b < n; b++)
                if (content[src][b]) acc[b] ^= (uint8_t)gf::mul(c, content[src][b]);
            step.src_ids.push_back(src);
            step.coef.push_back((uint8_t)c);
        }
        if (!any) return;
        step.dst_ids.push_back(dest);
        steps.push_back(std::move(step));
        content[dest] = std::move(acc);
        if (std::find(written.begin(), written.end(), dest) == written.end()) written.push_back(dest);
    }
};

}  // namespace

int plan_matrix_decode(int k, int m, const int* matrix, int row_k_ones, const int* erasures,
                       std::vector<LinearOp>& ops) {
    ops.clear();
    const int n = k + m;
    if (k < 1 || m < 1) return -1;
    // jerasure_erasures_to_erased
    std::vector<int> erased(n, 0);
    int alive = n;
    for (int i = 0; erasures[i] != -1; i++) {
        const int e = erasures[i];
        if (e < 0 || e >= n) return -1;
        if (!erased[e]) {
            erased[e] = 1;
            if (--alive < k) return -1;
        }
    }
    int lastdrive = k, edd = 0;
    for (int i = 0; i < k; i++)
        if (erased[i]) {
            edd++;
            lastdrive = i;
        }
    if (!row_k_ones || erased[k]) lastdrive = k;

    std::vector<int> dm_ids, decoding;
    if (edd > 1 || (edd > 0 && (!row_k_ones || erased[k]))) {
        for (int i = 0; (int)dm_ids.size() < k; i++)
            if (!erased[i]) dm_ids.push_back(i);
        std::vector<int> tmp((size_t)k * k, 0);
        for (int i = 0; i < k; i++) {
            if (dm_ids[i] < k) {
                tmp[(size_t)i * k + dm_ids[i]] = 1;
            } else {
                for (int j = 0; j < k; j++) tmp[(size_t)i * k + j] = matrix[(size_t)(dm_ids[i] - k) * k + j];
            }
        }
        if (invert_matrix(tmp, decoding, k) < 0) return -1;
    }

    Replay R(n);
    for (int i = 0; edd > 0 && i < lastdrive; i++) {
        if (erased[i]) {
            R.dotprod(k, &decoding[(size_t)i * k], dm_ids.data(), i);
            edd--;
        }
    }
    if (edd > 0) {
        std::vector<int> tmpids(k);
        for (int i = 0; i < k; i++) tmpids[i] = (i < lastdrive) ? i : i + 1;
        R.dotprod(k, matrix, tmpids.data(), lastdrive);
    }
    for (int i = 0; i < m; i++)
        if (erased[k + i]) R.dotprod(k, matrix + (size_t)i * k, nullptr, k + i);

    if (R.written.empty()) return 0;
    // Compose.  Valid iff no final content depends on the original bytes of a written block.
    std::vector<int> used(n, 0);
    bool composable = true;
    for (int w : R.written)
        for (int b = 0; b < n; b++)
            if (R.content[w][b]) {
                used[b] = 1;
                if (std::find(R.written.begin(), R.written.end(), b) != R.written.end()) composable = false;
            }
    if (!composable) {
        ops = std::move(R.steps);
        return 0;
    }
    LinearOp op;
    for (int b = 0; b < n; b++)
        if (used[b]) op.src_ids.push_back(b);
    for (int w : R.written) {
        op.dst_ids.push_back(w);
        for (int b : op.src_ids) op.coef.push_back(R.content[w][b]);
    }
    ops.push_back(std::move(op));
    return 0;
}

bool compose_chain(const std::vector<LinearOp>& ops, LinearOp& out) {
    // dense ids over the blocks the chain names
    std::vector<int> ids;
    for (const LinearOp& op : ops) {
        ids.insert(ids.end(), op.src_ids.begin(), op.src_ids.end());
        ids.insert(ids.end(), op.dst_ids.begin(), op.dst_ids.end());
    }
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const int n = (int)ids.size();
    auto at = [&](int id) { return (int)(std::lower_bound(ids.begin(), ids.end(), id) - ids.begin()); };
    // content[b]: block b's bytes as a combination of the ORIGINAL contents (identity until written)
    std::vector<std::vector<uint8_t>> content(n, std::vector<uint8_t>(n, 0));
    for (int b = 0; b < n; b++) content[b][b] = 1;
    std::vector<int> written;  // dense ids, first-write order
    std::vector<char> is_written(n, 0);
    std::vector<std::vector<uint8_t>> rows;
    for (const LinearOp& op : ops) {
        const int k = op.k_in(), m = op.m_out();
        if (op.coef.size() != (size_t)k * m) return false;
        rows.assign(m, std::vector<uint8_t>(n, 0));
        for (int p = 0; p < m; p++)  // every row reads the values before this op's writes
            for (int j = 0; j < k; j++) {
                const int c = op.coef[(size_t)p * k + j];
                if (!c) continue;
                const std::vector<uint8_t>& src = content[at(op.src_ids[j])];
                for (int b = 0; b < n; b++)
                    if (src[b]) rows[p][b] ^= (uint8_t)gf::mul(c, src[b]);
            }
        for (int p = 0; p < m; p++) {
            const int d = at(op.dst_ids[p]);
            content[d] = std::move(rows[p]);
            if (!is_written[d]) {
                is_written[d] = 1;
                written.push_back(d);
            }
        }
    }
    // one op over the original contents exists iff no written block's original bytes are read
    std::vector<char> used(n, 0);
    for (int w : written)
        for (int b = 0; b < n; b++)
            if (content[w][b]) {
                if (is_written[b]) return false;
                used[b] = 1;
            }
    LinearOp op;
    for (int b = 0; b < n; b++)
        if (used[b]) op.src_ids.push_back(ids[b]);
    if (op.src_ids.empty()) return false;  // every output zero: leave such a chain as it is
    op.coef.reserve(written.size() * op.src_ids.size());
    for (int w : written) {
        op.dst_ids.push_back(ids[w]);
        for (int b = 0; b < n; b++)
            if (used[b]) op.coef.push_back(content[w][b]);
    }
    out = std::move(op);
    return true;
}

std::shared_ptr<const std::vector<LinearOp>> encode_plan_cached(int k, int m, const int* matrix) {
    struct Entry {
        std::vector<int> key;
        std::shared_ptr<const std::vector<LinearOp>> ops;
    };
    thread_local std::unordered_map<uint64_t, std::vector<Entry>> cache;
    thread_local size_t entries = 0;
    thread_local std::vector<int> key;
    key.resize(2 + (size_t)k * m);
    key[0] = k;
    key[1] = m;
    std::copy(matrix, matrix + (size_t)k * m, key.begin() + 2);
    uint64_t h = 1469598103934665603ull;
    for (int x : key) h = (h ^ (uint32_t)x) * 1099511628211ull;
    auto& bucket = cache[h];
    for (const Entry& e : bucket)
        if (e.key == key) return e.ops;
    if (++entries > 1024) {  // bounded: a long-running caller sees an open set of partial matrices
        cache.clear();
        entries = 1;
    }
    auto ops = std::make_shared<std::vector<LinearOp>>();
    LinearOp op = plan_matrix_encode(k, m, matrix);
    if (op.m_out() > 0) ops->push_back(std::move(op));
    auto& b2 = cache[h];
    b2.push_back(Entry{key, ops});
    return b2.back().ops;
}

}  // namespace ecg
