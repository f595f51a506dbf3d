#!/bin/bash
# Builds tests/emu/libhyobfs_emu.so: the kernel + ABI sources compiled for the
# host CPU against hip_emu.h, with AddressSanitizer.  Test infrastructure only.
set -e
cd "$(dirname "$0")"
SRC=../../hysteria_amd/csrc
CXX=${CXX:-/opt/rocm/llvm/bin/clang++}
FLAGS="${EMU_EXTRA:-} -std=c++20 -O1 -g -fPIC -DHYOBFS_EMULATE -I. -I$SRC -x c++ -fsanitize=address -fno-omit-frame-pointer -pthread -Wno-unused-command-line-argument"
mkdir -p build
$CXX $FLAGS -c $SRC/salamander.hip -o build/salamander.o &
$CXX $FLAGS -c $SRC/hyobfs_api.cpp -o build/hyobfs_api.o &
$CXX $FLAGS -c $SRC/hyobfs_conn.cpp -o build/hyobfs_conn.o &
$CXX $FLAGS -c $SRC/conn_coalesce.cpp -o build/conn_coalesce.o &
$CXX $FLAGS -c $SRC/gecko.hip -o build/gecko.o &
$CXX $FLAGS -c $SRC/realm.hip -o build/realm.o &
$CXX $FLAGS -c $SRC/quic.hip -o build/quic.o &
$CXX $FLAGS -c $SRC/gecko_host.cpp -o build/gecko_host.o &
for n in $(seq 0 15); do $CXX $FLAGS -DHY_SW=$n -c $SRC/salamander_inst.hip -o build/inst_sw$n.o & done
wait
$CXX -shared -fsanitize=address -pthread -o ${EMU_OUT:-libhyobfs_emu.so} build/*.o
echo built tests/emu/libhyobfs_emu.so
