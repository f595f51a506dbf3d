#!/bin/bash
# Build an A/B variant of libhyobfs.so:
#   scripts/build_variant.sh NAME "-DFLAG=..." [PATCH ...]  ->  ab_builds/libhyobfs_NAME.so
# Extra compile flags go to every translation unit.  Each PATCH (a unified diff against
# hysteria_amd/csrc, e.g. tools/ab_patches/*.patch: ablations with wrong output, timing
# only) is applied to a scratch copy of the sources, so the product sources carry no
# ablation hooks.  ab_builds/ ships with every gpurun push: delete the variants once the
# A/B has run.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
FLAGS=${1:-}; shift || true
SRC=$R/hysteria_amd/csrc
if [ $# -gt 0 ]; then
  T=$(mktemp -d /tmp/hyvariant.XXXXXX)
  mkdir -p "$T/hysteria_amd" "$T/scripts"
  cp -r "$R/include" "$T/"
  mkdir -p "$T/hysteria_amd/csrc" && (cd "$SRC" && find . -maxdepth 1 -type f -exec cp {} "$T/hysteria_amd/csrc/" \;)
  cp "$R/scripts/src_sha.py" "$T/scripts/"
  for p in "$@"; do patch -s -d "$T/hysteria_amd/csrc" -p1 < "$p"; done
  SRC=$T/hysteria_amd/csrc
fi
mkdir -p "$R/ab_builds"
make -s -j8 -C "$SRC" BUILD="$R/ab_builds/$NAME" OUT="$R/ab_builds/libhyobfs_$NAME.so" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $FLAGS"
rm -rf "$R/ab_builds/$NAME"   # objects: only the .so travels to the GPU box
[ -n "${T:-}" ] && rm -rf "$T"
echo "$R/ab_builds/libhyobfs_$NAME.so"
