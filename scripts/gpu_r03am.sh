#!/bin/bash
# Round 3: packed wave kernel, groups taken in start order from an atomic counter (atom) against
# blockIdx order (main) on configs[2].
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03am
mkdir -p $O
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,atom=build_variants/libhyobfs_atom.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
echo done
