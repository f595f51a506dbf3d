#!/bin/bash
# Round 3: Gecko encode, chunks per lane in flight (HY_GK_U 2/4/6/8) and register caps.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03aa
mkdir -p $O
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,u8=build_variants/libhyobfs_u8.so,u8w5=build_variants/libhyobfs_u8w5.so,u6=build_variants/libhyobfs_u6.so,u2=build_variants/libhyobfs_u2.so" \
    timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
done
echo done
