#!/bin/bash
# Round 3: packed wave kernel, workgroups per launch (HYOBFS_WAVE_LAUNCH_BLOCKS; 4M bimodal = 32768
# workgroups), one process each; then packed GPU parity with 3-workgroup launches.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03al
mkdir -p $O
for B in 0 16384 8192 4096 2048 0; do
  HYOBFS_WAVE_LAUNCH_BLOCKS=$B AB_WORKLOAD=bimodal AB_ROUNDS=4 timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_B$B.txt 2>&1
done
HYOBFS_WAVE_LAUNCH_BLOCKS=3 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "packed or bimodal or ragged or shard or concurrent" > $O/pytest_blocks3.log 2>&1
echo done
