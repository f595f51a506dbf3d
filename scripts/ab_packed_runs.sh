#!/bin/bash
# Packed layout on the wave kernel with runs shorter than the 64-datagram group
# (HYOBFS_PACKED_RUN_LOG2): GPU parity under the forced wave kernel, then the
# bimodal bench for the default (persistent) kernel and each run length.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/packed_runs; mkdir -p $O
HYOBFS_KERNEL=wave HYOBFS_PACKED_RUN_LOG2=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_rl3.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python bench.py --workload bimodal --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $O/persistent_$r.json 2>>$O/err || exit 1
  for rl in 6 4 3 2; do
    HYOBFS_KERNEL=wave HYOBFS_PACKED_RUN_LOG2=$rl timeout -k 10 120 python bench.py --workload bimodal --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $O/wave_rl${rl}_$r.json 2>>$O/err || exit 1
  done
done
echo ok
