#!/bin/bash
# Round 3: tile kernel ablations, two interleaved processes per variant.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03c
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_main_$rep.txt 2>&1
  for v in align nobar pure ldplain stplain; do
    AB_NOCHECK=1 HYOBFS_LIB=build_variants/libhyobfs_$v.so timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_${v}_$rep.txt 2>&1
  done
done
echo done
