#!/bin/bash
# Round 3: pipelined packed kernel -- GPU parity under every kernel choice, bimodal A/B against the wave kernel.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  AB_WORKLOAD=bimodal timeout -k 10 300 python -u scripts/ab_variants.py auto,packed > $O/ab_bimodal_$rep.txt 2>&1
done
echo done
