#!/bin/bash
# Build an A/B variant of libhyobfs.so with extra compile flags:
#   scripts/build_variant.sh NAME "-DFLAG=..."  ->  build_variants/libhyobfs_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$R/build_variants"
make -s -j8 -C "$R/hysteria_amd/csrc" BUILD="$R/build_variants/$NAME" OUT="$R/build_variants/libhyobfs_$NAME.so" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $*"
echo "$R/build_variants/libhyobfs_$NAME.so"
