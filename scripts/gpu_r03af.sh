#!/bin/bash
# Round 3: packed wave kernel at 32 datagrams per wave (main): GPU parity of the packed cases,
# A/B against 64 per wave (d64) and against 64 park slots at 8 waves/SIMD (p64s).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "packed or bimodal or ragged or shard or concurrent" > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,d64=build_variants/libhyobfs_d64.so,p64s=build_variants/libhyobfs_p64s.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
echo done
