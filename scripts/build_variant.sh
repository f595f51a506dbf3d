#!/bin/bash
# Build an A/B variant of libhyobfs.so with extra compile flags:
#   scripts/build_variant.sh NAME "-DFLAG=..."  ->  ab_builds/libhyobfs_NAME.so
# ab_builds/ ships with every gpurun push: delete the variants once the A/B has run.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$R/ab_builds"
make -s -j8 -C "$R/hysteria_amd/csrc" BUILD="$R/ab_builds/$NAME" OUT="$R/ab_builds/libhyobfs_$NAME.so" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $*"
rm -rf "$R/ab_builds/$NAME"   # objects: only the .so travels to the GPU box
echo "$R/ab_builds/libhyobfs_$NAME.so"
