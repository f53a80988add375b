// Host-side coefficient-matrix construction and planning (tiny, k x k at most; SURVEY.md row a6:
// "keep on CPU").  These replace the matrix half of the Jerasure C API the reference links
// (CmakeLists.txt:116-134); the region (byte) half is the HIP engine.
#pragma once
#include <stdint.h>

#include <memory>
#include <vector>

namespace ecg {

// ---- Jerasure-equivalent matrix builders (w = 8).  Empty vector = failure / unsupported.
// reed_sol_vandermonde_coding_matrix(k, m, 8): rows k..k+m-1 of the systematic distribution
// matrix derived from the extended Vandermonde matrix (row 0 and column 0 all ones).
std::vector<int> reed_sol_vandermonde_coding_matrix(int k, int m);
// cauchy_good_general_coding_matrix(k, m, 8).  m == 2 selects Jerasure's hard-coded cbest_8 table,
// which is not available offline: returns empty (status ECG_EUNPINNED at the C ABI).
std::vector<int> cauchy_good_general_coding_matrix(int k, int m);
// The same two builders through a process-wide, mutex-protected cache keyed by (k, m): the facade's
// objects call them per operation (the reference rebuilds them per call, rs.cpp:22-23, lrc.cpp:27);
// entries are never dropped (at most one per distinct (k, m)), so the references stay valid.
const std::vector<int>& cached_vandermonde(int k, int m);
const std::vector<int>& cached_cauchy_good(int k, int m);
std::vector<int> cauchy_original_coding_matrix(int k, int m);
void cauchy_improve_coding_matrix(int k, int m, std::vector<int>& M);
int cauchy_n_ones(int e);
// jerasure_invert_matrix: in-place Gauss-Jordan on `mat` (destroyed), 0 or -1 (singular; `inv` then
// holds the state reached, as the library leaves it).
int invert_matrix(std::vector<int>& mat, std::vector<int>& inv, int rows);
// jerasure_matrix_multiply: (r1 x c1) * (r2 x c2) -> r1 x c2 (the library loops over r2).
std::vector<int> matrix_multiply(const int* m1, const int* m2, int r1, int c1, int r2, int c2);

// ---- Linear region operations over a block-id space.
// out[dst_ids[p]] = XOR_j coef[p * k_in + j] * in[src_ids[j]]   (GF(2^8), bytewise)
struct LinearOp {
    std::vector<int> src_ids;
    std::vector<int> dst_ids;
    std::vector<uint8_t> coef;  // m_out x k_in, row-major
    int k_in() const { return (int)src_ids.size(); }
    int m_out() const { return (int)dst_ids.size(); }
};

// jerasure_matrix_encode(k, m, matrix): data ids 0..k-1, coding ids k..k+m-1.  Rows that are all
// zero are omitted (jerasure_matrix_dotprod leaves such a destination untouched).
LinearOp plan_matrix_encode(int k, int m, const int* matrix);

// jerasure_matrix_decode(k, m, matrix, row_k_ones, erasures) replayed symbolically over GF(2^8):
// every dot product the library would execute is composed into one linear map from the blocks it
// reads to the blocks it writes (exact: the arithmetic is linear, no rounding), including the
// row_k_ones "last drive" shortcut and the re-encoding of erased coding blocks.  If a written block
// is ever read before it is written (not the case for any invertible pattern) the plan falls back to
// one op per library dot product.  Returns 0, or -1 exactly where the library returns -1
// (> m erasures, singular decoding matrix) or for erasure ids out of range.
int plan_matrix_decode(int k, int m, const int* matrix, int row_k_ones, const int* erasures,
                       std::vector<LinearOp>& ops);

// An op is BINARY when every coefficient is 0 or 1 (pure XOR network).
bool op_is_binary(const LinearOp& op);

// A chain of ops run in order (each op reads what its sources hold after the ops before it) as ONE op over
// the chain's original inputs: every block the chain writes, in first-write order, as its final linear
// combination of the blocks it reads before they are written (exact: substitution over GF(2^8)).  Sources
// are in ascending id order, columns that cancel to zero dropped.  false when no single op has the chain's
// effect: a block whose original bytes a final value depends on is also written (the kernel would read it
// while other workgroups write it), or every final value is zero.
bool compose_chain(const std::vector<LinearOp>& ops, LinearOp& out);

// plan_matrix_encode through a per-thread cache keyed by (k, m, matrix entries): the same plan object
// for the same matrix, so per-stripe calls neither rebuild it nor copy it into a batch scope.
std::shared_ptr<const std::vector<LinearOp>> encode_plan_cached(int k, int m, const int* matrix);

}  // namespace ecg
