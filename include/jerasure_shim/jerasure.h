/* Drop-in replacement for Jerasure 2.0's jerasure.h (w = 8 subset the reference uses), backed by libecg.
 *
 * hhlgt/erasure-codes-prototype includes "jerasure.h", "reed_sol.h" and "cauchy.h"
 * (project/include/ec/erasure_code.h:3-5) and links `Jerasure gf_complete` (project/CmakeLists.txt:116-134).
 * Putting this directory first on the include path and linking libecg instead routes every byte of
 * jerasure_matrix_encode / jerasure_matrix_decode / galois_region_xor to the MI355X kernels, with
 * Jerasure's signatures, return values and buffer semantics (include/ecg.h tier 1).
 *
 * Differences from the library, all on failure paths Jerasure does not have: a HIP error (or w != 8) is
 * reported on stderr in the reference's print-and-continue style (rs.cpp:30-41); matrix builders return
 * NULL where Jerasure would abort or the cbest_8 table is needed (cauchy.h). */
#ifndef ECG_JERASURE_SHIM_H
#define ECG_JERASURE_SHIM_H

#include <stdio.h>

#include "../ecg.h"
#include "galois.h"

static inline void ecg_shim_report(int rc, const char* fn) {
    if (rc < 0 && rc != ECG_EUNDECODABLE)
        fprintf(stderr, "[libecg] %s failed (%d): %s\n", fn, rc, rc == ECG_EHIP ? ecg_last_error() : "bad arguments");
}

/* jerasure.h: void jerasure_matrix_encode(int k, int m, int w, int *matrix, char **data_ptrs,
 *                                         char **coding_ptrs, int size); */
static inline void jerasure_matrix_encode(int k, int m, int w, int* matrix, char** data_ptrs, char** coding_ptrs,
                                          int size) {
    ecg_shim_report(ecg_jerasure_matrix_encode(k, m, w, matrix, data_ptrs, coding_ptrs, size),
                    "jerasure_matrix_encode");
}

/* int jerasure_matrix_decode(...): 0 on success, -1 if the erasures cannot be decoded. */
static inline int jerasure_matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures,
                                         char** data_ptrs, char** coding_ptrs, int size) {
    const int rc = ecg_jerasure_matrix_decode(k, m, w, matrix, row_k_ones, erasures, data_ptrs, coding_ptrs, size);
    ecg_shim_report(rc, "jerasure_matrix_decode");
    return rc < 0 ? -1 : 0;
}

static inline void jerasure_matrix_dotprod(int k, int w, int* matrix_row, int* src_ids, int dest_id,
                                           char** data_ptrs, char** coding_ptrs, int size) {
    ecg_shim_report(ecg_jerasure_matrix_dotprod(k, w, matrix_row, src_ids, dest_id, data_ptrs, coding_ptrs, size),
                    "jerasure_matrix_dotprod");
}

/* int jerasure_invert_matrix(int *mat, int *inv, int rows, int w): 0, or -1 if singular. */
static inline int jerasure_invert_matrix(int* mat, int* inv, int rows, int w) {
    return ecg_jerasure_invert_matrix(mat, inv, rows, w);
}

/* int *jerasure_matrix_multiply(...): malloc'd r1 x c2 product (the caller frees it). */
static inline int* jerasure_matrix_multiply(int* m1, int* m2, int r1, int c1, int r2, int c2, int w) {
    return ecg_jerasure_matrix_multiply(m1, m2, r1, c1, r2, c2, w);
}

#endif
