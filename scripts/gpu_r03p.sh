#!/bin/bash
# Round 3: packed wave kernel with the one-pass look-back scan -- GPU parity, A/B against the prepass scan (prev), bench.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo done
