#!/bin/bash
# Round 3: tile kernel v2 (key wave + 3 data waves) parity + A/B variants.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tile" --timeout 120 --timeout-method thread > $O/pytest_tile.log 2>&1
timeout -k 10 300 python -u scripts/ab_kernels.py wave,tile > $O/ab_main.txt 2>&1
AB_NOCHECK=1 HYOBFS_LIB=build_variants/libhyobfs_nohash.so timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_nohash.txt 2>&1
HYOBFS_LIB=build_variants/libhyobfs_u6.so timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_u6.txt 2>&1
HYOBFS_LIB=build_variants/libhyobfs_u9.so timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_u9.txt 2>&1
timeout -k 10 300 python -u scripts/ab_kernels.py tile,wave > $O/ab_main2.txt 2>&1
echo done
