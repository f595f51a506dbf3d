#!/bin/bash
# Round 3: packed layout -- GPU parity of the packed cases; bimodal A/B of main (one-launch
# chunked look-back scan) against prev (tile sums + one-workgroup scan) and three ablation builds
# of main (no boundary step / no hash / neither; wrong output, timing only).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "packed or bimodal or ragged or shard" > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so,nobound!=build_variants/libhyobfs_nobound.so,nohash!=build_variants/libhyobfs_nohash.so,nobh!=build_variants/libhyobfs_nobh.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
echo done
