// Host-side GF(2^8) arithmetic for matrix construction (product code, not the oracle).
// Field: GF(2^8) with primitive polynomial x^8+x^4+x^3+x^2+1 (0x11d), gf-complete's w=8 default
// that the reference selects through Jerasure with w = 8 (erasure_code.h:65).
// Implemented with log / antilog tables over the generator 2; the byte hot path never uses these,
// it runs in the HIP kernels (gf_kernels.hip).
#pragma once
#include <stdint.h>

namespace ecg {
namespace gf {

struct Tables {
    uint8_t exp[512];
    int16_t log[256];
    Tables() {
        int x = 1;
        for (int i = 0; i < 255; i++) {
            exp[i] = (uint8_t)x;
            exp[i + 255] = (uint8_t)x;
            log[x] = (int16_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11d;
        }
        exp[510] = exp[0];
        exp[511] = exp[1];
        log[0] = -1;
    }
};

inline const Tables& tables() {
    static const Tables t;
    return t;
}

inline int mul(int a, int b) {
    a &= 0xff;
    b &= 0xff;
    if (a == 0 || b == 0) return 0;
    const Tables& t = tables();
    return t.exp[t.log[a] + t.log[b]];
}

inline int inv(int a) {
    const Tables& t = tables();
    a &= 0xff;
    if (a == 0) return 0;
    return t.exp[255 - t.log[a]];
}

// galois_single_divide semantics: 0 if a == 0, -1 if b == 0.
inline int div(int a, int b) {
    if ((a & 0xff) == 0) return 0;
    if ((b & 0xff) == 0) return -1;
    return mul(a, inv(b));
}

}  // namespace gf
}  // namespace ecg
