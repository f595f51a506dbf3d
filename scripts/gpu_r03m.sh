#!/bin/bash
# Round 3: Gecko encode (wave-group kernel) occupancy / register variants, in-process A/B.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gecko.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gecko.log 2>&1
V=build_variants
L="main=hysteria_amd/libhyobfs.so"
for n in gku2 gku8 gkwpe5 gkwpe6 gkwpe8 gkpsw5 gkpsw6; do L="$L,$n=$V/libhyobfs_$n.so"; done
for rep in 1 2; do
  AB_LIBS="$L" timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
done
echo done
