#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 60 ./tools/glds_probe > $O/glds_probe.json 2>&1
HYOBFS_LIB=build_variants/libhyobfs_stage.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -k "tile" --timeout 120 --timeout-method thread > $O/pytest_tile_stage.log 2>&1 || true
export AB_LIBS="main=hysteria_amd/libhyobfs.so,ldplain=build_variants/libhyobfs_ldplain.so,stage=build_variants/libhyobfs_stage.so,stagent=build_variants/libhyobfs_stagent.so"
for rep in 1 2 3; do
  timeout -k 10 300 python -u scripts/ab_variants.py tile > $O/ab_$rep.txt 2>&1
done
echo done
