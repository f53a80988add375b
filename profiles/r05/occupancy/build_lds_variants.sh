#!/bin/bash
# Tuning builds for the occupancy probe (never shipped): libecg with every kernel launched with N bytes of
# unused dynamic LDS, so at most floor(160 KiB / N) workgroups share a CU.  The product source is not edited:
# gf_kernels.hip is copied into the build directory with launch_kernel's shared-memory argument replaced.
#   profiles/r05/occupancy/build_lds_variants.sh 16384 20480 ...  -> erasure-codes-prototype_amd/lib/libecg_ldsN.so
set -euo pipefail
cd "$(dirname "$0")/../../.."
PKG=$PWD/erasure-codes-prototype_amd
HIPCC=/opt/rocm/bin/hipcc
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Wno-unused-result"
for n in "$@"; do
  obj=$PKG/build/variant_lds$n
  mkdir -p $obj
  grep -c 'return hipLaunchKernel((const void\*)kernel, grid, block, argv, 0, st);' $PKG/csrc/gf_kernels.hip > /dev/null
  sed "s|return hipLaunchKernel((const void\*)kernel, grid, block, argv, 0, st);|return hipLaunchKernel((const void*)kernel, grid, block, argv, $n, st);|" \
    $PKG/csrc/gf_kernels.hip > $obj/gf_kernels.hip
  cp $PKG/csrc/*.hpp $obj/
  $HIPCC $CXXFLAGS --offload-arch=gfx950 -mcode-object-version=5 -I$PKG/csrc -c $obj/gf_kernels.hip -o $obj/gf_kernels.o &
  for f in matrix engine codes planning capi; do
    [ -f $PKG/build/variant_lds_common/$f.o ] || { mkdir -p $PKG/build/variant_lds_common &&
      $HIPCC $CXXFLAGS -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $PKG/csrc/$f.cpp -o $PKG/build/variant_lds_common/$f.o; }
  done
  wait
  $HIPCC -shared -fPIC --offload-arch=gfx950 -o $PKG/lib/libecg_lds$n.so $obj/gf_kernels.o $PKG/build/variant_lds_common/*.o \
    -Wl,-soname,libecg_lds$n.so
  echo "lib/libecg_lds$n.so"
done
