#!/bin/bash
# Engine concurrency under ThreadSanitizer (CPU only, no GPU): libecg's host translation units and the host
# side of gf_kernels.hip (--offload-host-only: no device code), linked with tests/tsan/hip_stub.cpp -- a CPU
# stand-in for the HIP runtime that emulates the library's kernels bit-exactly -- and the driver
# tests/tsan/engine_race.cpp (8 threads of random proxy-like calls, every result against the oracle).
#   tools/tsan_host.sh [variant] [threads] [ops] [seed]
# variant "seeded" builds engine.cpp with -DECG_TEST_TSAN_SEEDED_RACE (retire() without its lock): the
# run must then report a data race.  Variant "sharedkey" builds it with -DECG_TEST_PER_THREAD_SHARED_KEY
# (round 4's retirement keying of hipStreamPerThread): the run must then report a device-time hazard in its
# per-thread scenario (the stub's check that no table a pending launch reads is rewritten from another
# stream).  tests/test_sanitize.py checks all three.
set -euo pipefail
cd "$(dirname "$0")/.."
PKG=erasure-codes-prototype_amd
VARIANT=${1:-product}
OBJ=$PKG/build/tsan_$VARIANT
mkdir -p "$OBJ"
CXX=/opt/rocm/lib/llvm/bin/clang++
CC=/opt/rocm/lib/llvm/bin/clang
HIPCC=/opt/rocm/bin/hipcc
FLAGS="-O1 -g -fPIC -fsanitize=thread -fno-omit-frame-pointer -Wall -Wno-unused-parameter -Wno-unused-value -Wno-unused-result"
INC="-D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$PKG/csrc"
EXTRA=""
[ "$VARIANT" = seeded ] && EXTRA="-DECG_TEST_TSAN_SEEDED_RACE"
[ "$VARIANT" = sharedkey ] && EXTRA="-DECG_TEST_PER_THREAD_SHARED_KEY"
pids=()
for f in matrix engine codes planning capi; do
  $CXX $FLAGS -std=c++17 $INC $EXTRA -x c++ -c $PKG/csrc/$f.cpp -o $OBJ/$f.o &
  pids+=($!)
done
# its warnings (device-only attributes seen host-side) go to a log, printed if the compile fails
( $HIPCC $FLAGS -std=c++17 --offload-arch=gfx950 --offload-host-only -c $PKG/csrc/gf_kernels.hip -o $OBJ/gf_kernels.o \
    2>"$OBJ/gf_kernels.log" || { echo "tsan_host.sh: host-only compile of gf_kernels.hip failed:" >&2; cat "$OBJ/gf_kernels.log" >&2; exit 1; } ) &
pids+=($!)
$CXX $FLAGS -std=c++17 $INC -c tests/tsan/hip_stub.cpp -o $OBJ/hip_stub.o &
pids+=($!)
$CXX $FLAGS -std=c++17 $INC -c tests/tsan/engine_race.cpp -o $OBJ/engine_race.o &
pids+=($!)
$CC $FLAGS -std=c11 -mavx2 -c oracle/jerasure_w8.c -o $OBJ/oracle.o &
pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
# the kernel file's fat-binary symbol points at the stub's empty stand-in (no device code is loaded)
FATBIN=$(nm -u $OBJ/gf_kernels.o | awk '/__hip_fatbin_/{print $2}')
$CXX -fsanitize=thread -o $OBJ/engine_race $OBJ/*.o -Wl,--defsym,$FATBIN=hip_stub_fatbin -lpthread
TSAN_OPTIONS="halt_on_error=0 exitcode=66 second_deadlock_stack=1 history_size=4 ${TSAN_OPTIONS:-}" \
  "$OBJ/engine_race" "${2:-8}" "${3:-150}" "${4:-1}"
