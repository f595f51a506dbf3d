#!/bin/bash
# Round 3: wave kernel sweep with unconditional loads (exact vmcnt waits) -- GPU parity of
# the wave-kernel cases, A/B against prev (conditional loads) on configs[2] and on the
# uniform batch under the wave kernel.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so" \
  timeout -k 10 300 python -u scripts/ab_variants.py wave,tile > $O/ab_uniform.txt 2>&1
echo done
