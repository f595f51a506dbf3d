#!/bin/bash
# Round 3: packed wave kernel, batch-size sweep on the bimodal mix (tail effect: a fixed
# cost per launch shows as a per-datagram time that falls with P).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03t
mkdir -p $O
for P in 1048576 2097152 4194304 8388608 16777216; do
  AB_WORKLOAD=bimodal AB_ROUNDS=4 timeout -k 10 300 python -u scripts/ab_variants.py auto 0 $P > $O/ab_bimodal_P$P.txt 2>&1
done
echo done
