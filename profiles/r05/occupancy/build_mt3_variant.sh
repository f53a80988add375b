#!/bin/bash
# Tuning build (never shipped): the single-output LDS pad (ECG_OPT_MT1_LDS_PAD) applied to launches of up to
# 3 outputs, so the option can be swept over k -> 2 and k -> 3 shapes (shapes_probe.py, ECG_PROBE_M).  The
# product source is not edited.  -> erasure-codes-prototype_amd/lib/libecg_padmt3.so
set -euo pipefail
cd "$(dirname "$0")/../../.."
PKG=$PWD/erasure-codes-prototype_amd
HIPCC=/opt/rocm/bin/hipcc
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Wno-unused-result"
obj=$PKG/build/variant_padmt3
mkdir -p $obj
python3 - "$PKG/csrc/gf_kernels.hip" "$obj/gf_kernels.hip" <<'PY'
import sys
src = open(sys.argv[1]).read()
old = "    const unsigned lds = MT == 1 ? mt1_lds_pad(a.k) : 0u;"
assert src.count(old) == 1
open(sys.argv[2], "w").write(src.replace(old, "    const unsigned lds = MT <= 3 ? mt1_lds_pad(a.k) : 0u;"))
PY
cp $PKG/csrc/*.hpp $obj/
$HIPCC $CXXFLAGS --offload-arch=gfx950 -mcode-object-version=5 -I$PKG/csrc -c $obj/gf_kernels.hip -o $obj/gf_kernels.o
for f in matrix engine codes planning capi; do
  $HIPCC $CXXFLAGS -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $PKG/csrc/$f.cpp -o $obj/$f.o &
done
wait
$HIPCC -shared -fPIC --offload-arch=gfx950 -o $PKG/lib/libecg_padmt3.so $obj/*.o -Wl,-soname,libecg_padmt3.so
echo lib/libecg_padmt3.so
