#!/bin/bash
# Round 3: packed wave kernel, datagrams per wave (HY_PACKED_DPW 64 shipped / 32 / 16) and
# hash ablations (d16nh, d64nh: wrong output) on configs[2].
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ae
mkdir -p $O
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,d32=build_variants/libhyobfs_d32.so,d16=build_variants/libhyobfs_d16.so,d16nh!=build_variants/libhyobfs_d16nh.so,d64nh!=build_variants/libhyobfs_d64nh.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
echo done
