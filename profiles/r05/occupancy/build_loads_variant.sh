#!/bin/bash
# Tuning build (never shipped): the vector kernel's "every input load in flight before the first fold" block,
# which only single calls (GF_MODE_INLINE_LAT) take, enabled for every mode (batched strided and
# pointer-table launches too) for k <= 16.  The product source is not edited: gf_kernels.hip is copied into the
# build directory with that one condition changed.  -> erasure-codes-prototype_amd/lib/libecg_allloads.so
set -euo pipefail
cd "$(dirname "$0")/../../.."
PKG=$PWD/erasure-codes-prototype_amd
HIPCC=/opt/rocm/bin/hipcc
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Wno-unused-result"
obj=$PKG/build/variant_allloads
mkdir -p $obj
python3 - "$PKG/csrc/gf_kernels.hip" "$obj/gf_kernels.hip" <<'PY'
import sys
src = open(sys.argv[1]).read()
old = "        if constexpr (MODE == GF_MODE_INLINE_LAT) {\n            // uniform: every load in flight"
assert src.count(old) == 1
open(sys.argv[2], "w").write(src.replace(old, "        if constexpr (true) {\n            // uniform: every load in flight"))
PY
cp $PKG/csrc/*.hpp $obj/
$HIPCC $CXXFLAGS --offload-arch=gfx950 -mcode-object-version=5 -I$PKG/csrc -c $obj/gf_kernels.hip -o $obj/gf_kernels.o
for f in matrix engine codes planning capi; do
  $HIPCC $CXXFLAGS -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $PKG/csrc/$f.cpp -o $obj/$f.o &
done
wait
$HIPCC -shared -fPIC --offload-arch=gfx950 -o $PKG/lib/libecg_allloads.so $obj/*.o -Wl,-soname,libecg_allloads.so
echo lib/libecg_allloads.so
