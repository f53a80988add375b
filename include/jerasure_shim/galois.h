/* Drop-in for gf-complete-era Jerasure galois.h: the one symbol the reference uses (lrc.cpp:1511,2140),
 * backed by libecg (include/ecg.h).  void galois_region_xor(char *src, char *dest, int nbytes): dest ^= src. */
#ifndef ECG_GALOIS_SHIM_H
#define ECG_GALOIS_SHIM_H

#include <stdio.h>

#include "../ecg.h"

static inline void galois_region_xor(char* src, char* dest, int nbytes) {
    const int rc = ecg_galois_region_xor(src, dest, nbytes);
    if (rc < 0) fprintf(stderr, "[libecg] galois_region_xor failed (%d): %s\n", rc, ecg_last_error());
}

#endif
