#!/bin/bash
# Round 3, first GPU session: tile kernel parity + in-process A/B against the wave kernel.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 120 ./tools/region_copy > $O/region_copy.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tile" --timeout 120 --timeout-method thread > $O/pytest_tile.log 2>&1
timeout -k 10 300 python -u scripts/ab_kernels.py wave,tile > $O/ab_main.txt 2>&1
AB_NOCHECK=1 HYOBFS_LIB=build_variants/libhyobfs_nohash.so timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_nohash.txt 2>&1
HYOBFS_LIB=build_variants/libhyobfs_u4.so timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_u4.txt 2>&1
echo done
