#!/bin/bash
# Round 3: Gecko encode sweep with unconditional loads (exact vmcnt waits, padding stores
# before message stores) -- Gecko GPU tests, A/B against prev (shipped) and a 5-wave cap.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k gecko > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so,wpe5=build_variants/libhyobfs_wpe5.so" \
    timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
done
echo done
