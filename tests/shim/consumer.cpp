// Reference-shaped consumer of include/jerasure_shim/: calls the seven Jerasure symbols with the argument
// shapes hhlgt/erasure-codes-prototype uses, through the shim headers only, linked against libecg.so.
//   consumer matrices                      -> prints the matrix builders' / invert / multiply results (CPU)
//   consumer bytes IN OUT k m B            -> reads k*B data bytes from IN, writes to OUT:
//        m coding blocks (rs.cpp:22-24: zeroed outputs, proxy.cpp:335-342),
//        the 2 blocks rebuilt by jerasure_matrix_decode after erasing data 0 and coding 1
//          (rs.cpp:34-36: row_k_ones = failed_num, erased buffers hold garbage),
//        1 partial-decoding block for failure 0 from survivors 1..k (erasure_code.cpp:113-150:
//          invert F[survivors], multiply by F[failures], encode the columns of the first half),
//        data 1 after galois_region_xor(data 0, data 1)  (lrc.cpp:1511 shape).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cauchy.h"
#include "jerasure.h"
#include "reed_sol.h"

static void print_matrix(const char* name, const int* M, int rows, int cols) {
    printf("%s", name);
    for (int i = 0; i < rows * cols; i++) printf(" %d", M ? M[i] : -1);
    printf("\n");
}

static int matrices() {
    int* rs = reed_sol_vandermonde_coding_matrix(10, 4, 8);
    print_matrix("rs_10_4", rs, 4, 10);
    int* cg = cauchy_good_general_coding_matrix(12, 3, 8);
    print_matrix("cauchy_good_12_3", cg, 3, 12);
    // erasure_code.cpp:122-131: F = [I; M] rows of the survivors, inverted, then multiplied
    const int k = 4, m = 2;
    int* M = reed_sol_vandermonde_coding_matrix(k, m, 8);
    std::vector<int> F((size_t)(k + m) * k, 0);
    for (int i = 0; i < k; i++) F[(size_t)i * k + i] = 1;
    memcpy(&F[(size_t)k * k], M, sizeof(int) * k * m);
    const int surv[4] = {1, 2, 3, 4}, fail[1] = {0};
    std::vector<int> S((size_t)k * k), inv((size_t)k * k), Ff((size_t)k);
    for (int i = 0; i < k; i++) memcpy(&S[(size_t)i * k], &F[(size_t)surv[i] * k], sizeof(int) * k);
    memcpy(Ff.data(), &F[(size_t)fail[0] * k], sizeof(int) * k);
    const int rc = jerasure_invert_matrix(S.data(), inv.data(), k, 8);
    printf("invert_rc %d\n", rc);
    print_matrix("inverse", inv.data(), k, k);
    int* R = jerasure_matrix_multiply(Ff.data(), inv.data(), 1, k, k, k, 8);
    print_matrix("decode_row", R, 1, k);
    free(R);
    free(M);
    free(cg);
    free(rs);  // rs.cpp:17: the reference frees the builder's result with free()
    return 0;
}

static int bytes(const char* in_path, const char* out_path, int k, int m, int B) {
    std::vector<char> data((size_t)k * B), coding((size_t)m * B, 0);
    FILE* f = fopen(in_path, "rb");
    if (!f || fread(data.data(), 1, data.size(), f) != data.size()) return 2;
    fclose(f);
    std::vector<char*> dp(k), cp(m);
    for (int i = 0; i < k; i++) dp[i] = &data[(size_t)i * B];
    for (int i = 0; i < m; i++) cp[i] = &coding[(size_t)i * B];
    int* M = reed_sol_vandermonde_coding_matrix(k, m, 8);
    jerasure_matrix_encode(k, m, 8, M, dp.data(), cp.data(), B);
    std::vector<char> coded = coding;
    // decode: lose data 0 and coding 1, garbage in both
    std::vector<char> d2 = data, c2 = coding;
    std::vector<char*> dp2(k), cp2(m);
    for (int i = 0; i < k; i++) dp2[i] = &d2[(size_t)i * B];
    for (int i = 0; i < m; i++) cp2[i] = &c2[(size_t)i * B];
    memset(dp2[0], 0x3c, B);
    memset(cp2[1], 0x3c, B);
    int erasures[3] = {0, k + 1, -1};
    const int failed_num = 2;
    const int drc = jerasure_matrix_decode(k, m, 8, M, failed_num, erasures, dp2.data(), cp2.data(), B);
    // partial decoding of failure 0 from survivors 1..k (coding 0 = block k), local = survivors 1..k/2
    std::vector<int> F((size_t)(k + m) * k, 0);
    for (int i = 0; i < k; i++) F[(size_t)i * k + i] = 1;
    memcpy(&F[(size_t)k * k], M, sizeof(int) * k * m);
    std::vector<int> Sm((size_t)k * k), inv((size_t)k * k);
    for (int i = 0; i < k; i++) memcpy(&Sm[(size_t)i * k], &F[(size_t)(i + 1) * k], sizeof(int) * k);
    jerasure_invert_matrix(Sm.data(), inv.data(), k, 8);
    int* R = jerasure_matrix_multiply(&F[0], inv.data(), 1, k, k, k, 8);
    const int nloc = k / 2;
    std::vector<int> Rl(R, R + nloc);
    std::vector<char> part(B, 0);
    char* pp[1] = {part.data()};
    std::vector<char*> loc(nloc);
    for (int i = 0; i < nloc; i++) loc[i] = (i + 1 < k) ? dp[i + 1] : cp[i + 1 - k];
    jerasure_matrix_encode(nloc, 1, 8, Rl.data(), loc.data(), pp, B);
    free(R);
    // galois_region_xor(src, dest, n)
    std::vector<char> x0(data.begin(), data.begin() + B), x1(data.begin() + B, data.begin() + 2 * (size_t)B);
    galois_region_xor(x0.data(), x1.data(), B);
    free(M);
    FILE* o = fopen(out_path, "wb");
    if (!o) return 2;
    fwrite(coded.data(), 1, coded.size(), o);
    fwrite(dp2[0], 1, B, o);
    fwrite(cp2[1], 1, B, o);
    fwrite(part.data(), 1, B, o);
    fwrite(x1.data(), 1, B, o);
    fclose(o);
    printf("decode_rc %d\n", drc);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && !strcmp(argv[1], "matrices")) return matrices();
    if (argc >= 7 && !strcmp(argv[1], "bytes")) return bytes(argv[2], argv[3], atoi(argv[4]), atoi(argv[5]), atoi(argv[6]));
    fprintf(stderr, "usage: consumer matrices | consumer bytes IN OUT k m B\n");
    return 2;
}
