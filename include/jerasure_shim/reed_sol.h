/* Drop-in for Jerasure's reed_sol.h (the symbol the reference uses: rs.cpp:7,34,297; lrc.cpp:624,935,1170),
 * backed by libecg.  Returns a malloc'd m x k matrix (the reference frees it, rs.cpp:17), NULL if k + m > 256
 * or w != 8. */
#ifndef ECG_REED_SOL_SHIM_H
#define ECG_REED_SOL_SHIM_H

#include "jerasure.h"

static inline int* reed_sol_vandermonde_coding_matrix(int k, int m, int w) {
    return ecg_reed_sol_vandermonde_coding_matrix(k, m, w);
}

#endif
