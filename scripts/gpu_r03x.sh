#!/bin/bash
# Round 3: Gecko encode, message-count sweep (launch tail: a fixed cost shows as a
# per-frame time that falls with the batch).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03x
mkdir -p $O
for M in 131072 262144 524288 1048576; do
  AB_MSGS=$M AB_ROUNDS=4 timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_M$M.txt 2>&1
done
echo done
