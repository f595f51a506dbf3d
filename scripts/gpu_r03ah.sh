#!/bin/bash
# Round 3: tile kernel rate by batch size (1M / 4M / 8M x 1200 B; 8M is the per-GPU shard of
# configs[3] that bench.py runs for N > 1), one process each.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ah
mkdir -p $O
for P in 1048576 4194304 8388608; do
  AB_ROUNDS=4 timeout -k 10 300 python -u scripts/ab_variants.py tile 1200 $P > $O/ab_tile_P$P.txt 2>&1
done
echo done
