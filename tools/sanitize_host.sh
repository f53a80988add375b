#!/bin/bash
# Host-code sanitizer run (CPU only, no GPU): every host translation unit of libecg plus
# tests/sanitize/host_fuzz.cpp built with AddressSanitizer + UndefinedBehaviorSanitizer. Device code is
# never sanitized: the host-only lines carry -fno-gpu-sanitize, and the HIP file is compiled for its host
# side only (--offload-host-only, as tools/tsan_host.sh does). The fuzz driver runs the CPU-only ABI
# surface and launches no kernel, so the kernel file's fat-binary symbol points at an empty stand-in
# instead of a gfx950 code object (that device compile took most of this script's three minutes).
set -euo pipefail
cd "$(dirname "$0")/.."
PKG=erasure-codes-prototype_amd
OBJ=$PKG/build/sanitize
mkdir -p "$OBJ"
HIPCC=/opt/rocm/bin/hipcc
CXX="-O1 -g -std=c++17 -fPIC -Wall -Wno-unused-parameter -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
# the translation units compile in parallel; every status is checked
pids=()
for f in matrix engine codes planning capi; do
  $HIPCC $CXX -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $PKG/csrc/$f.cpp -o $OBJ/$f.o &
  pids+=($!)
done
( $HIPCC $CXX --offload-arch=gfx950 --offload-host-only -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize \
    -c $PKG/csrc/gf_kernels.hip -o $OBJ/gf_kernels.o 2>"$OBJ/gf_kernels.log" ||
  { echo "sanitize_host.sh: host-only compile of gf_kernels.hip failed:" >&2; cat "$OBJ/gf_kernels.log" >&2; exit 1; } ) &
pids+=($!)
printf 'const char ecg_no_device_code[16] = {0};\n' > $OBJ/no_device_code.c
gcc -c $OBJ/no_device_code.c -o $OBJ/no_device_code.o
$HIPCC $CXX -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$PKG/csrc -c tests/sanitize/host_fuzz.cpp -o $OBJ/host_fuzz.o &
pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
FATBIN=$(nm -u $OBJ/gf_kernels.o | awk '/__hip_fatbin_/{print $2}')
$HIPCC -o $OBJ/host_fuzz $OBJ/*.o -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize \
  -Wl,--defsym,$FATBIN=ecg_no_device_code
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OBJ/host_fuzz"
