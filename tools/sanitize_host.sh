#!/bin/bash
# Host-code sanitizer run (CPU only, no GPU): every host translation unit of libecg plus
# tests/sanitize/host_fuzz.cpp built with AddressSanitizer + UndefinedBehaviorSanitizer. Device code is
# never sanitized: the host-only lines carry -fno-gpu-sanitize, the HIP file takes the flags through
# -Xarch_host. The fuzz driver then runs the CPU-only ABI surface.
set -euo pipefail
cd "$(dirname "$0")/.."
PKG=erasure-codes-prototype_amd
OBJ=$PKG/build/sanitize
mkdir -p "$OBJ"
HIPCC=/opt/rocm/bin/hipcc
CXX="-O1 -g -std=c++17 -fPIC -Wall -Wno-unused-parameter -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
# the translation units compile in parallel (the HIP one takes longest); every status is checked
pids=()
for f in matrix engine codes planning capi; do
  $HIPCC $CXX -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $PKG/csrc/$f.cpp -o $OBJ/$f.o &
  pids+=($!)
done
$HIPCC $CXX --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -c $PKG/csrc/gf_kernels.hip -o $OBJ/gf_kernels.o &
pids+=($!)
$HIPCC $CXX -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$PKG/csrc -c tests/sanitize/host_fuzz.cpp -o $OBJ/host_fuzz.o &
pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC -o $OBJ/host_fuzz $OBJ/*.o --offload-arch=gfx950 -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OBJ/host_fuzz"
