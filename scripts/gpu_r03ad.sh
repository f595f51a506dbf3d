#!/bin/bash
# Round 3: packed wave kernel, datagrams per run (HYOBFS_PACKED_RUN_LOG2 6/5/4/3), one process each.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ad
mkdir -p $O
for rl in 6 5 4 3 6; do
  HYOBFS_PACKED_RUN_LOG2=$rl AB_WORKLOAD=bimodal AB_ROUNDS=4 timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_rl$rl.txt 2>&1
done
echo done
