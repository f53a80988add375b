#!/bin/bash
# Tuning builds (never shipped): tools/build_variant.sh NAME "-DMACRO=V ..." -> erasure-codes-prototype_amd/lib/libecg_NAME.so
set -euo pipefail
name=$1; flags=$2
cd "$(dirname "$0")/../erasure-codes-prototype_amd"
obj=build/variant_$name
mkdir -p "$obj" lib
HIPCC=/opt/rocm/bin/hipcc
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Wno-unused-result"
$HIPCC $CXXFLAGS --offload-arch=gfx950 -mcode-object-version=5 $flags -c csrc/gf_kernels.hip -o $obj/gf_kernels.o
for f in csrc/matrix.cpp csrc/engine.cpp csrc/codes.cpp csrc/planning.cpp csrc/capi.cpp; do
  $HIPCC $CXXFLAGS -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $flags -c $f -o $obj/$(basename $f .cpp).o
done
$HIPCC -shared -fPIC --offload-arch=gfx950 -o lib/libecg_$name.so $obj/*.o -Wl,-soname,libecg.so
echo "lib/libecg_$name.so"
