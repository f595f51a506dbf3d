#!/bin/bash
# Round 3: packed wave kernel on configs[2] -- ablations (wrong output, timing only):
# no boundary loads in step 3, 16-aligned sweep loads, both; temporal sweep loads; a
# control build identical to main.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03u
mkdir -p $O
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,ctl=build_variants/libhyobfs_prev.so,nobload!=build_variants/libhyobfs_nobload.so,alignld!=build_variants/libhyobfs_alignld.so,both!=build_variants/libhyobfs_both.so,tload=build_variants/libhyobfs_tload.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
echo done
