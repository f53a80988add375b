#!/bin/bash
# Build and run tools/host_cost.cpp (host cost of the per-stripe facade path) against the HIP stand-in in no-op
# mode: libecg's host translation units + the host side of gf_kernels.hip + loopback/replay.cpp + tests/tsan/hip_stub.cpp,
# -O2 (PROF=1 adds -pg and writes a gprof report).  CPU only.
#   tools/host_cost.sh [batches] [stripes]
set -euo pipefail
cd "$(dirname "$0")/.."
PKG=erasure-codes-prototype_amd
OBJ=$PKG/build/host_cost
mkdir -p "$OBJ"
CXX=/opt/rocm/lib/llvm/bin/clang++
HIPCC=/opt/rocm/bin/hipcc
PG=""
[ "${PROF:-0}" = 1 ] && PG="-pg"
FLAGS="-O2 -g -fPIC $PG -Wno-unused-result"
INC="-D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$PKG/csrc"
pids=()
for f in matrix engine codes planning capi; do
  $CXX $FLAGS -std=c++17 $INC -x c++ -c $PKG/csrc/$f.cpp -o $OBJ/$f.o & pids+=($!)
done
( $HIPCC $FLAGS -std=c++17 --offload-arch=gfx950 --offload-host-only -c $PKG/csrc/gf_kernels.hip -o $OBJ/gf_kernels.o \
    2>"$OBJ/gf_kernels.log" || { cat "$OBJ/gf_kernels.log" >&2; exit 1; } ) & pids+=($!)
$CXX $FLAGS -std=c++17 $INC -c tests/tsan/hip_stub.cpp -o $OBJ/hip_stub.o & pids+=($!)
$CXX $FLAGS -std=c++17 $INC -c $PKG/loopback/replay.cpp -o $OBJ/replay.o & pids+=($!)
$CXX $FLAGS -std=c++17 $INC -c tools/host_cost.cpp -o $OBJ/host_cost_main.o & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
FATBIN=$(nm -u $OBJ/gf_kernels.o | awk '/__hip_fatbin_/{print $2}')
$CXX $PG -o $OBJ/host_cost $OBJ/*.o -Wl,--defsym,$FATBIN=hip_stub_fatbin -lpthread
cd $OBJ && HIP_STUB_NOOP=1 ./host_cost "${1:-200}" "${2:-256}"
if [ "${PROF:-0}" = 1 ]; then gprof -b -p ./host_cost gmon.out | head -40; fi
