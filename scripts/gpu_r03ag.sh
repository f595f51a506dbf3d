#!/bin/bash
# Round 3: Gecko aligned sweep, independent binary search per chunk (gkbs: pipelined, 5-wave cap;
# gkbs6: 6-wave cap; gkbsnp: unpipelined, 6 waves) against main (carried forward walk).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ag
mkdir -p $O
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,gkbs=build_variants/libhyobfs_gkbs.so,gkbs6=build_variants/libhyobfs_gkbs6.so,gkbsnp=build_variants/libhyobfs_gkbsnp.so" \
    timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
done
echo done
