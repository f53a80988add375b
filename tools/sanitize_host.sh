#!/bin/bash
# Host-code sanitizer run (CPU only, no GPU): every host translation unit of libecg plus
# tests/sanitize/host_fuzz.cpp built with -fsanitize=address,undefined (device code untouched: the HIP
# file gets the flags through -Xarch_host only), then the fuzz driver runs the CPU-only ABI surface.
set -euo pipefail
cd "$(dirname "$0")/.."
PKG=erasure-codes-prototype_amd
OBJ=$PKG/build/sanitize
mkdir -p "$OBJ"
HIPCC=/opt/rocm/bin/hipcc
SAN="-fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
CXX="-O1 -g -std=c++17 -fPIC -Wall -Wno-unused-parameter"
for f in matrix engine codes planning capi; do
  $HIPCC $CXX $SAN -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $PKG/csrc/$f.cpp -o $OBJ/$f.o
done
$HIPCC $CXX --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -c $PKG/csrc/gf_kernels.hip -o $OBJ/gf_kernels.o
$HIPCC $CXX $SAN -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -c tests/sanitize/host_fuzz.cpp \
  -o $OBJ/host_fuzz.o
$HIPCC -o $OBJ/host_fuzz $OBJ/*.o --offload-arch=gfx950 -fsanitize=address -fsanitize=undefined
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OBJ/host_fuzz"
