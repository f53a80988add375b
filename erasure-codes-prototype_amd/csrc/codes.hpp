// ErasureCode facade: the reference's EC class hierarchy (project/include/ec/{erasure_code,rs,lrc,pc}.h)
// re-expressed over the GPU engine.  Same class names, method names, argument meaning and index
// conventions; every method compiles its work into LinearOps over the call's block space
// (data_ptrs ++ coding_ptrs) and runs them in ONE engine call, so multi-step methods (product-code
// encode / iterative decode) keep intermediate blocks in HBM.  Byte work never runs on the CPU.
//
// Differences from the reference, all deliberate:
//   * methods return int status instead of void (the reference prints and returns);
//   * blocks may be host (reference semantics) or device pointers (`mem`, `stream`);
//   * coding matrices come from a process-wide (k, m) cache instead of being rebuilt per call
//     (rs.cpp:22-23); the objects keep no lazily-filled state, so concurrent calls on one object are
//     safe as long as its parameters are not changed meanwhile.
// Partitioning (placement of a stripe's blocks over clusters) and repair planning (which helper blocks each
// cluster contributes to a partial-decoding repair) are host logic in planning.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/ecg.h"
#include "matrix.hpp"

namespace ecg {

using CodingParameters = ecg_coding_parameters;

// erasure_code.h:53-58.  help_blocks[i] = the blocks one cluster (partition) contributes.
struct RepairPlan {
    bool local_or_column = false;
    std::vector<int> failure_idxs;
    std::vector<std::vector<int>> help_blocks;
};

// A call's work: ops over block ids, ids index `blocks` (data_ptrs then coding_ptrs).
struct Plan {
    std::vector<LinearOp> ops;
};
using SharedOps = std::shared_ptr<const std::vector<LinearOp>>;

// Sub-call helpers (ids of the sub-call's data / coding blocks inside the caller's block space).
void append_encode(Plan& plan, int k, int m, const int* matrix, const std::vector<int>& data_ids,
                   const std::vector<int>& coding_ids);
int append_decode(Plan& plan, int k, int m, const int* matrix, int row_k_ones, const int* erasures,
                  const std::vector<int>& data_ids, const std::vector<int>& coding_ids);

class ErasureCode {
public:
    int k = 6;
    int m = 3;
    int w = 8;
    bool local_or_column = false;
    int mem = ECG_MEM_HOST;
    hipStream_t stream = nullptr;

    ErasureCode() = default;
    ErasureCode(int k_, int m_) : k(k_), m(m_) {}
    virtual ~ErasureCode() = default;

    virtual void init_coding_parameters(const CodingParameters& cp);
    virtual void get_coding_parameters(CodingParameters& cp) const;

    virtual int encode(char** data_ptrs, char** coding_ptrs, int block_size) = 0;
    virtual int decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) = 0;
    virtual int check_if_decodable(const std::vector<int>& failure_idxs) = 0;  // 1, 0, or < 0
    virtual int make_encoding_matrix(int* final_matrix) = 0;
    int encode_partial_blocks_for_encoding(char** data_ptrs, char** coding_ptrs, int block_size,
                                           std::vector<int> data_idxs, std::vector<int> parity_idxs);
    int encode_partial_blocks_for_decoding(char** data_ptrs, char** coding_ptrs, int block_size,
                                           std::vector<int> local_survivor_idxs, std::vector<int> survivor_idxs,
                                           std::vector<int> failure_idxs);
    int perform_addition(char** data_ptrs, char** coding_ptrs, int block_size, int block_num, int parity_num);
    // The main proxy's two steps of a partial-decoding repair (handle_repair.cpp:371-376) in one pass:
    // out[u] = (encode_partial_blocks_for_decoding over local_ptrs)[u] XOR perform_addition over
    // partial_ptrs (n_partials = cnt * f, interleaved like perform_addition's input).  Reads each local
    // block and each helper partial once and writes the f outputs once (the separate calls also write
    // and re-read the main proxy's own f partials).  local_survivor_idxs may be empty.
    int encode_partial_blocks_for_decoding_with_addition(char** local_ptrs, char** partial_ptrs, int n_partials,
                                                         char** out_ptrs, int block_size,
                                                         std::vector<int> local_survivor_idxs,
                                                         std::vector<int> survivor_idxs, std::vector<int> failure_idxs);
    // The same for stripe merging: the parity proxy's own encode_partial_blocks_for_encoding over its data
    // blocks plus perform_addition with the helpers' partial parities (handle_merge.cpp:159,319).
    int encode_partial_blocks_for_encoding_with_addition(char** local_ptrs, char** partial_ptrs, int n_partials,
                                                         char** out_ptrs, int block_size, std::vector<int> data_idxs,
                                                         std::vector<int> parity_idxs);

    // The coefficient matrix (n_out x n_in) a partial call applies (erasure_code.cpp:97-150 semantics).
    virtual int partial_encoding_matrix(std::vector<int> data_idxs, std::vector<int> parity_idxs,
                                        std::vector<int>& out) = 0;
    virtual int partial_decoding_matrix(std::vector<int> local_survivor_idxs, std::vector<int> survivor_idxs,
                                        std::vector<int> failure_idxs, std::vector<int>& out) = 0;

    virtual std::string self_information() const = 0;

    // Everything the coefficient matrices of this object depend on (class + parameters, sub-codes
    // included): the key of the per-thread plan cache of the per-call methods.  A class that adds a
    // matrix-relevant field appends it here.
    virtual void state_key(std::vector<int>& key) const;

    // ---- partitioning and repair planning (planning.cpp)
    int placement_rule = ECG_PLACE_OPTIMAL;  // erasure_code.h:66 default OPTIMAL
    std::vector<std::vector<int>> partition_plan;
    virtual void partition_flat();
    virtual void partition_random() = 0;
    virtual void partition_optimal() = 0;
    virtual int partition_sub_optimal() { return ECG_EINVAL; }  // Azu_LRC only
    int generate_partition();  // erasure_code.cpp:159-169 (+ ECG_PLACE_SUB_OPTIMAL)
    // 1 = plans generated, 0 = undecodable (the reference's bool), < 0 = bad arguments
    virtual int generate_repair_plan(const std::vector<int>& failure_idxs, std::vector<RepairPlan>& plans) = 0;
    void set_random_seed(uint64_t seed) {
        rng_ = seed;
        rng_seeded_ = true;
    }

    // erasure_code.cpp:30-61
    static void get_full_matrix(int* matrix, int kk);
    static void make_submatrix_by_rows(int cols, const int* matrix, int* new_matrix, const std::vector<int>& idxs);
    static void make_submatrix_by_cols(int cols, int rows, const int* matrix, int* new_matrix,
                                       const std::vector<int>& idxs);
    // erasure_code.cpp:97-111 / 113-150 as matrices
    static void partial_encoding_matrix_(int k_, const int* full_matrix, const std::vector<int>& data_idxs,
                                         const std::vector<int>& parity_idxs, std::vector<int>& out);
    static void partial_decoding_matrix_(int k_, const int* full_matrix, const std::vector<int>& local_survivor_idxs,
                                         const std::vector<int>& survivor_idxs,
                                         const std::vector<int>& failure_idxs, std::vector<int>& out);

protected:
    // random_range / random_index (utils.cpp:6-21): the reference draws from a fresh random_device-seeded
    // mt19937 per call; here a per-object splitmix64 stream (seeded from random_device, or explicitly for
    // reproducible placements).  Same support, uniform.
    uint64_t rng_ = 0;
    bool rng_seeded_ = false;
    uint64_t next_random();
    int random_range(int lo, int hi);
    int random_index(int len);

    // Execute a plan over data_ptrs (n_data) ++ coding_ptrs (n_coding) on this object's memory tier.
    int run(const Plan& plan, char** data_ptrs, int n_data, char** coding_ptrs, int n_coding, long long B);
    // The same with an interned plan (per-thread plan caches below): recorded in a batch scope without a copy.
    int run(const SharedOps& ops, char** data_ptrs, int n_data, char** coding_ptrs, int n_coding, long long B);
    // jerasure_matrix_encode / _decode over this call's pointers
    int run_encode(int kk, int mm, const int* matrix, char** data_ptrs, char** coding_ptrs, long long B,
                   bool stable_matrix = false);
    int run_with_addition(const std::vector<int>& R, int nl, int nf, char** local_ptrs, char** partial_ptrs,
                          int n_partials, char** out_ptrs, long long B);
    int run_decode(int kk, int mm, const int* matrix, int row_k_ones, int* erasures, char** data_ptrs,
                   char** coding_ptrs, long long B);
};

// ------------------------------------------------------------------ RS (rs.h / rs.cpp)
class RSCode : public ErasureCode {
public:
    RSCode() = default;
    RSCode(int k_, int m_) : ErasureCode(k_, m_) {}
    int encode(char** data_ptrs, char** coding_ptrs, int block_size) override;
    int decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;
    int make_encoding_matrix(int* final_matrix) override;
    int partial_encoding_matrix(std::vector<int> data_idxs, std::vector<int> parity_idxs,
                                std::vector<int>& out) override;
    int partial_decoding_matrix(std::vector<int> lsi, std::vector<int> si, std::vector<int> fi,
                                std::vector<int>& out) override;
    std::string self_information() const override;

    void partition_random() override;   // rs.cpp:78-101
    void partition_optimal() override;  // rs.cpp:103-116
    void help_blocks_for_single_block_repair_oneoff(int failure_idx, std::vector<std::vector<int>>& help_blocks);
    void help_blocks_for_multi_blocks_repair_oneoff(const std::vector<int>& failure_idxs,
                                                    std::vector<std::vector<int>>& help_blocks);
    int generate_repair_plan(const std::vector<int>& failure_idxs, std::vector<RepairPlan>& plans) override;

    // Plans over an arbitrary id space (used by the product codes)
    int plan_encode(Plan& p, const std::vector<int>& data_ids, const std::vector<int>& coding_ids);
    int plan_decode(Plan& p, const std::vector<int>& data_ids, const std::vector<int>& coding_ids, int* erasures,
                    int failed_num);
    std::vector<int> full_matrix();  // [I_k ; M]

protected:
    const std::vector<int>& vandermonde();  // reed_sol_vandermonde_coding_matrix(k, m), cached process-wide
};

class EnlargedRSCode : public RSCode {
public:
    int x = 2;
    int seri_num = 1;
    EnlargedRSCode() = default;
    EnlargedRSCode(int k_, int m_) : RSCode(k_, m_) {}
    void init_coding_parameters(const CodingParameters& cp) override;
    void state_key(std::vector<int>& key) const override;
    int make_encoding_matrix(int* final_matrix) override;
    std::string self_information() const override;
};

// ------------------------------------------------------------------ LRC family (lrc.h / lrc.cpp)
class LocallyRepairableCode : public ErasureCode {
public:
    int l = 0, g = 0, r = 0;
    LocallyRepairableCode() = default;
    LocallyRepairableCode(int k_, int l_, int g_) : ErasureCode(k_, l_ + g_), l(l_), g(g_) {
        r = l_ > 0 ? (k_ + l_ - 1) / l_ : 0;
    }
    void init_coding_parameters(const CodingParameters& cp) override;
    void get_coding_parameters(CodingParameters& cp) const override;
    void state_key(std::vector<int>& key) const override;
    int encode(char** data_ptrs, char** coding_ptrs, int block_size) override;
    int decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) override;
    int decode_global(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num);
    int decode_local(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num,
                     int group_id);
    int check_if_decodable(const std::vector<int>& failure_idxs) override;
    int partial_encoding_matrix(std::vector<int> data_idxs, std::vector<int> parity_idxs,
                                std::vector<int>& out) override;
    int partial_decoding_matrix(std::vector<int> lsi, std::vector<int> si, std::vector<int> fi,
                                std::vector<int>& out) override;

    virtual int make_group_matrix(int* group_matrix, int group_id, int size) = 0;  // 1 x size
    virtual int get_group_size(int group_id, int& min_idx) = 0;
    virtual int bid2gid(int block_id) = 0;
    virtual int idxingroup(int block_id) = 0;

    virtual void grouping_information(std::vector<std::vector<int>>& groups) = 0;
    void partition_random() override;   // lrc.cpp:215-238
    void partition_optimal() override {}  // lrc.h:75
    virtual void help_blocks_for_single_block_repair_oneoff(int failure_idx,
                                                            std::vector<std::vector<int>>& help_blocks);
    void help_blocks_for_multi_blocks_repair_oneoff(const std::vector<int>& failure_idxs,
                                                    std::vector<std::vector<int>>& help_blocks);
    int generate_repair_plan(const std::vector<int>& failure_idxs, std::vector<RepairPlan>& plans) override;

protected:
    std::vector<int> full_matrix();                        // [I_k ; G ; L]
    std::vector<int> group_full_matrix(int group_size, int group_id);  // [I_gs ; group row]
    virtual int remap_local(int idx, int group_size, int min_idx) const;
    virtual bool cauchy_based() const { return false; }
};

class Azu_LRC : public LocallyRepairableCode {
public:
    Azu_LRC(int k_, int l_, int g_) : LocallyRepairableCode(k_, l_, g_) { r = l_ > 0 ? (k_ + l_ - 1) / l_ : 0; }
    int make_encoding_matrix(int* final_matrix) override;
    int make_group_matrix(int* group_matrix, int group_id, int size) override;
    int get_group_size(int group_id, int& min_idx) override;
    int bid2gid(int block_id) override;
    int idxingroup(int block_id) override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;
    std::string self_information() const override;
    void grouping_information(std::vector<std::vector<int>>& groups) override;  // lrc.cpp:706-723
    void partition_optimal() override;                                            // lrc.cpp:725-814
    int partition_sub_optimal() override;                                         // lrc.cpp:816-873
};

class Azu_LRC_1 : public LocallyRepairableCode {
public:
    Azu_LRC_1(int k_, int l_, int g_) : LocallyRepairableCode(k_, l_, g_) { r = l_ > 1 ? (k_ + l_ - 2) / (l_ - 1) : 0; }
    int make_encoding_matrix(int* final_matrix) override;
    int make_group_matrix(int* group_matrix, int group_id, int size) override;
    int get_group_size(int group_id, int& min_idx) override;
    int bid2gid(int block_id) override;
    int idxingroup(int block_id) override;
    std::string self_information() const override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;      // lrc.cpp:881-931
    void grouping_information(std::vector<std::vector<int>>& groups) override;  // lrc.cpp:1051-1069
    void partition_optimal() override;                                            // lrc.cpp:1071-1088
};

class Opt_LRC : public LocallyRepairableCode {
public:
    Opt_LRC(int k_, int l_, int g_) : LocallyRepairableCode(k_, l_, g_) { r = l_ > 0 ? (k_ + g_ + l_ - 1) / l_ : 0; }
    int make_encoding_matrix(int* final_matrix) override;
    int make_group_matrix(int* group_matrix, int group_id, int size) override;
    int get_group_size(int group_id, int& min_idx) override;
    int bid2gid(int block_id) override;
    int idxingroup(int block_id) override;
    std::string self_information() const override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;      // lrc.cpp:1096-1166
    void grouping_information(std::vector<std::vector<int>>& groups) override;  // lrc.cpp:1270-1282
    void partition_optimal() override;                                            // lrc.cpp:1284-1301
};

class Opt_Cau_LRC : public LocallyRepairableCode {
public:
    Opt_Cau_LRC(int k_, int l_, int g_) : LocallyRepairableCode(k_, l_, g_) { r = l_ > 0 ? (k_ + l_ - 1) / l_ : 0; }
    int make_encoding_matrix(int* final_matrix) override;
    int make_group_matrix(int* group_matrix, int group_id, int size) override;
    int get_group_size(int group_id, int& min_idx) override;
    int bid2gid(int block_id) override;
    int idxingroup(int block_id) override;
    std::string self_information() const override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;      // lrc.cpp:1415-1483
    void grouping_information(std::vector<std::vector<int>>& groups) override;  // lrc.cpp:1641-1658
    void partition_optimal() override;                                            // lrc.cpp:1660-1749
    void help_blocks_for_single_block_repair_oneoff(int failure_idx,
                                                    std::vector<std::vector<int>>& help_blocks) override;
    int generate_repair_plan(const std::vector<int>& failure_idxs, std::vector<RepairPlan>& plans) override;
    int surviving_group_id = 0;  // lrc.h:171 (uninitialised in the reference; only read after being set)

protected:
    int remap_local(int idx, int group_size, int min_idx) const override;
    bool cauchy_based() const override { return true; }
};

class Uni_Cau_LRC : public LocallyRepairableCode {
public:
    Uni_Cau_LRC(int k_, int l_, int g_) : LocallyRepairableCode(k_, l_, g_) { r = l_ > 0 ? (k_ + g_ + l_ - 1) / l_ : 0; }
    int make_encoding_matrix(int* final_matrix) override;
    int make_group_matrix(int* group_matrix, int group_id, int size) override;
    int get_group_size(int group_id, int& min_idx) override;
    int bid2gid(int block_id) override;
    int idxingroup(int block_id) override;
    std::string self_information() const override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;      // lrc.cpp:2025-2095
    void grouping_information(std::vector<std::vector<int>>& groups) override;  // lrc.cpp:2273-2285
    void partition_optimal() override;                                            // lrc.cpp:2287-2304

protected:
    bool cauchy_based() const override { return true; }
};

// ------------------------------------------------------------------ Product codes (pc.h / pc.cpp)
class ProductCode : public ErasureCode {
public:
    RSCode row_code, col_code;
    int k1 = 0, m1 = 0, k2 = 0, m2 = 0;
    ProductCode() = default;
    ProductCode(int k1_, int m1_, int k2_, int m2_)
        : ErasureCode(k1_ * k2_, (k1_ + m1_) * (k2_ + m2_) - k1_ * k2_), row_code(k1_, m1_), col_code(k2_, m2_),
          k1(k1_), m1(m1_), k2(k2_), m2(m2_) {}
    void init_coding_parameters(const CodingParameters& cp) override;
    void get_coding_parameters(CodingParameters& cp) const override;
    void state_key(std::vector<int>& key) const override;
    int encode(char** data_ptrs, char** coding_ptrs, int block_size) override;
    int decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;
    int make_encoding_matrix(int*) override { return ECG_OK; }  // pc.h:37: empty
    int partial_encoding_matrix(std::vector<int> data_idxs, std::vector<int> parity_idxs,
                                std::vector<int>& out) override;
    int partial_decoding_matrix(std::vector<int> lsi, std::vector<int> si, std::vector<int> fi,
                                std::vector<int>& out) override;
    std::string self_information() const override;

    int rowcol2bid(int row, int col) const;
    void bid2rowcol(int bid, int& row, int& col) const;
    virtual int oldbid2newbid_for_merge(int old_block_id, int x, int seri_num, bool isvertical);

    void partition_flat() override;     // pc.cpp:378-388
    void partition_random() override;   // pc.cpp:390-421
    void partition_optimal() override;  // pc.cpp:423-443
    int generate_repair_plan(const std::vector<int>& failure_idxs, std::vector<RepairPlan>& plans) override;

protected:
    virtual RSCode& rowc() { return row_code; }  // code used for rows in encode/decode
    virtual RSCode& colc() { return col_code; }
    virtual RSCode& partial_col() { return col_code; }  // code used by partial calls (local_or_column)
    virtual RSCode& partial_row() { return row_code; }
    virtual bool has_global() const { return true; }
    int plan_iterative_decode(Plan& plan, int* erasures, int failed_num, int ncols, int nrows);
    // plan_iterative_decode through the per-thread call-plan cache, composed (codes.cpp finish_plan), and run
    int decode_iterative(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num,
                         int ncols, int nrows);
    std::vector<std::vector<int>> block_map() const;  // [row][col] -> block id in data ++ coding space
};

class HPC : public ProductCode {
public:
    EnlargedRSCode e_row_code, e_col_code;
    bool isvertical = true;
    HPC(int k1_, int m1_, int k2_, int m2_) : ProductCode(k1_, m1_, k2_, m2_), e_row_code(k1_, m1_), e_col_code(k2_, m2_) {}
    void init_coding_parameters(const CodingParameters& cp) override;
    int oldbid2newbid_for_merge(int old_block_id, int x, int seri_num, bool isvertical) override;
    std::string self_information() const override;
    void state_key(std::vector<int>& key) const override;

protected:
    RSCode& rowc() override { return isvertical ? (RSCode&)row_code : (RSCode&)e_row_code; }
    RSCode& colc() override { return isvertical ? (RSCode&)e_col_code : (RSCode&)col_code; }
    RSCode& partial_col() override { return isvertical ? (RSCode&)e_col_code : (RSCode&)col_code; }
    RSCode& partial_row() override { return isvertical ? (RSCode&)row_code : (RSCode&)e_row_code; }
};

class HVPC : public ProductCode {
public:
    HVPC(int k1_, int m1_, int k2_, int m2_) : ProductCode(k1_, m1_, k2_, m2_) { m = k1_ * m2_ + k2_ * m1_; }
    void init_coding_parameters(const CodingParameters& cp) override;
    int encode(char** data_ptrs, char** coding_ptrs, int block_size) override;
    int decode(char** data_ptrs, char** coding_ptrs, int block_size, int* erasures, int failed_num) override;
    int check_if_decodable(const std::vector<int>& failure_idxs) override;
    std::string self_information() const override;
    void partition_random() override;   // pc.cpp:1091-1129
    void partition_optimal() override;  // pc.cpp:1131-1158

protected:
    bool has_global() const override { return false; }
};

// metadata.cpp:48-77
ErasureCode* ec_factory(int ec_type, const CodingParameters& cp);

}  // namespace ecg
