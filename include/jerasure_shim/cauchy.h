/* Drop-in for Jerasure's cauchy.h (symbols used by the reference: lrc.cpp:1487,1522,1576,2099,2160,2215),
 * backed by libecg.  cauchy_good_general_coding_matrix(k, 2, 8) returns NULL: Jerasure answers it from its
 * hard-coded cbest_8 table, which is not available offline; the library never guesses. */
#ifndef ECG_CAUCHY_SHIM_H
#define ECG_CAUCHY_SHIM_H

#include "jerasure.h"

static inline int* cauchy_original_coding_matrix(int k, int m, int w) { return ecg_cauchy_original_coding_matrix(k, m, w); }
static inline void cauchy_improve_coding_matrix(int k, int m, int w, int* matrix) {
    ecg_cauchy_improve_coding_matrix(k, m, w, matrix);
}
static inline int* cauchy_good_general_coding_matrix(int k, int m, int w) {
    return ecg_cauchy_good_general_coding_matrix(k, m, w);
}
static inline int cauchy_n_ones(int n, int w) { return ecg_cauchy_n_ones(n, w); }

#endif
