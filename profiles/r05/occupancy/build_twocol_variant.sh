#!/bin/bash
# Tuning build (never shipped): batched vector launches (not single calls) process TWO 16-byte columns per
# lane per iteration -- every load of both columns' input group issued before either fold -- so a wave keeps
# twice the bytes in flight, at a lower occupancy hint (ECG_OCC_OVERRIDE, default 4 here: <= 128 VGPRs) and
# so fewer workgroups, i.e. fewer open block streams, per CU.  The product source is not edited: gf_kernels.hip
# is patched into the build directory.   build_twocol_variant.sh [occ] -> lib/libecg_twocol<occ>.so
set -euo pipefail
cd "$(dirname "$0")/../../.."
OCC=${1:-4}
PKG=$PWD/erasure-codes-prototype_amd
HIPCC=/opt/rocm/bin/hipcc
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Wno-unused-result"
obj=$PKG/build/variant_twocol$OCC
mkdir -p $obj
python3 - "$PKG/csrc/gf_kernels.hip" "$obj/gf_kernels.hip" <<'PY'
import sys
src = open(sys.argv[1]).read()
old = "    for (long long c = c0 + threadIdx.x; c < c1; c += kThreads) {\n        const long long off = c << 4;\n"
assert src.count(old) == 1
new = '''    if constexpr (MODE != GF_MODE_INLINE_LAT) {
        for (long long c = c0 + threadIdx.x; c < c1; c += 2 * kThreads) {
            const bool two = c + kThreads < c1;
            const long long off0 = c << 4, off1 = two ? (c + kThreads) << 4 : off0;
            uint32_t acc0[MT][4], acc1[MT][4];
#pragma unroll
            for (int p = 0; p < MT; ++p)
#pragma unroll
                for (int d = 0; d < 4; ++d) acc0[p][d] = acc1[p][d] = 0u;
            int j = 0;
            for (; j + 4 <= k; j += 4) {
                uint32_t x0[4][4], x1[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off0, x0[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off1, x1[u]);
                fold<MT, 4, BIN>(x0, T + (size_t)j * MT, acc0);
                fold<MT, 4, BIN>(x1, T + (size_t)j * MT, acc1);
            }
            if (j + 2 <= k) {
                uint32_t x0[2][4], x1[2][4];
#pragma unroll
                for (int u = 0; u < 2; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off0, x0[u]);
#pragma unroll
                for (int u = 0; u < 2; ++u) load16<NT>(src_ptr<MODE>(a, s, prog, j + u) + off1, x1[u]);
                fold<MT, 2, BIN>(x0, T + (size_t)j * MT, acc0);
                fold<MT, 2, BIN>(x1, T + (size_t)j * MT, acc1);
                j += 2;
            }
            if (j < k) {
                uint32_t x0[1][4], x1[1][4];
                load16<NT>(src_ptr<MODE>(a, s, prog, j) + off0, x0[0]);
                load16<NT>(src_ptr<MODE>(a, s, prog, j) + off1, x1[0]);
                fold<MT, 1, BIN>(x0, T + (size_t)j * MT, acc0);
                fold<MT, 1, BIN>(x1, T + (size_t)j * MT, acc1);
            }
#pragma unroll
            for (int p = 0; p < MT; ++p)
                if (p < nrows) {
                    store16<NT>(dst[p] + off0, acc0[p]);
                    if (two) store16<NT>(dst[p] + off1, acc1[p]);
                }
        }
        return;
    }
''' + old
open(sys.argv[2], "w").write(src.replace(old, new))
PY
cp $PKG/csrc/*.hpp $obj/
$HIPCC $CXXFLAGS --offload-arch=gfx950 -mcode-object-version=5 -DECG_OCC_OVERRIDE=$OCC -I$PKG/csrc -c $obj/gf_kernels.hip -o $obj/gf_kernels.o
for f in matrix engine codes planning capi; do
  $HIPCC $CXXFLAGS -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $PKG/csrc/$f.cpp -o $obj/$f.o &
done
wait
$HIPCC -shared -fPIC --offload-arch=gfx950 -o $PKG/lib/libecg_twocol$OCC.so $obj/*.o -Wl,-soname,libecg_twocol$OCC.so
echo lib/libecg_twocol$OCC.so
