#!/bin/bash
# Round 3: where the ragged-layout tile kernels spend their time -- in-process
# A/B of build variants and ablations (Gecko encode; packed Salamander bimodal).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03l
mkdir -p $O
V=build_variants
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,gkwave=$V/libhyobfs_gkwave.so,gku4=$V/libhyobfs_gku4.so,nopad!=$V/libhyobfs_gknopad.so,nohash!=$V/libhyobfs_gknohash.so" \
    timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
  AB_LIBS="main=hysteria_amd/libhyobfs.so,pt16k=$V/libhyobfs_pt16k.so,pt0=$V/libhyobfs_pt0.so,nohash!=$V/libhyobfs_gknohash.so" \
    AB_WORKLOAD=bimodal timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
echo done
