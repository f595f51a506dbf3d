#!/bin/bash
# Builds tests/emu/libhyobfs_emu.so: the kernel + ABI sources compiled for the
# host CPU against hip_emu.h, with AddressSanitizer.  Test infrastructure only.
set -e
cd "$(dirname "$0")"
SRC=../../hysteria_amd/csrc
CXX=${CXX:-/opt/rocm/llvm/bin/clang++}
FLAGS="${EMU_EXTRA:-} -std=c++20 -O1 -g -fPIC -DHYOBFS_EMULATE -I. -I$SRC -x c++ -fsanitize=address -fno-omit-frame-pointer -pthread -Wno-unused-command-line-argument"
mkdir -p build
rm -f build/*.o
pids=()
for f in salamander.hip hyobfs_api.cpp hyobfs_conn.cpp conn_coalesce.cpp gecko.hip realm.hip quic.hip gecko_host.cpp; do
  $CXX $FLAGS -c $SRC/$f -o build/${f%.*}.o & pids+=($!)
done
for n in $(seq 0 15); do $CXX $FLAGS -DHY_SW=$n -c $SRC/salamander_inst.hip -o build/inst_sw$n.o & pids+=($!); done
for p in "${pids[@]}"; do wait "$p" || { echo "emulated build: a compile failed" >&2; exit 1; }; done
$CXX -shared -fsanitize=address -pthread -o ${EMU_OUT:-libhyobfs_emu.so} build/*.o
echo built tests/emu/libhyobfs_emu.so
