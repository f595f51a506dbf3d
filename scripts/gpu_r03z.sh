#!/bin/bash
# Round 3: Gecko encode ablations (wrong output, timing only): no padding keystream,
# no key hash, no edge chunks, none of the three; main = shipped.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03z
mkdir -p $O
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,noks!=build_variants/libhyobfs_noks.so,nohash!=build_variants/libhyobfs_nohash.so,noedge!=build_variants/libhyobfs_noedge.so,none!=build_variants/libhyobfs_none.so" \
    timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
done
echo done
