#!/bin/bash
# Round 3: tile kernel, tiles per launch (HYOBFS_TILE_LAUNCH_TILES) on 1M and 8M x 1200 B, one process each.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ak
mkdir -p $O
for P in 1048576 8388608; do
  for T in 65536 32768 16384 8192 65536; do
    HYOBFS_TILE_LAUNCH_TILES=$T AB_ROUNDS=4 timeout -k 10 300 python -u scripts/ab_variants.py tile 1200 $P > $O/ab_P${P}_T$T.txt 2>&1
  done
done
echo done
