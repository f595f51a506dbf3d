#!/bin/bash
# Wave kernel: parked boundary chunks (shipped) vs the boundary-free sweep
# (HYOBFS_KERNEL=flat) on 1M x 1200 B, two processes; counters of the flat
# kernel; then the GPU tests (every parity case also runs under flat).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/flat; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  step ab_$i 240 python -u scripts/ab_kernels.py wave,flat > $O/ab_$i.txt 2>&1
done
step pytest 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_one.py uniform 5 flat
done
echo done
