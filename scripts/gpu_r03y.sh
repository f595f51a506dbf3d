#!/bin/bash
# Round 3: Gecko encode, a workgroup per 64-frame group (quad keys, edges a thread per
# (frame, candidate), four waves sweep quarters) -- Gecko GPU tests, A/B against prev
# (a wave per group) and register caps of 6 and 7 waves/SIMD; message-count sweep.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k gecko > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so,wpe6=build_variants/libhyobfs_wpe6.so,wpe7=build_variants/libhyobfs_wpe7.so" \
    timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
done
AB_MSGS=1048576 AB_ROUNDS=3 AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so" \
  timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_M1048576.txt 2>&1
echo done
