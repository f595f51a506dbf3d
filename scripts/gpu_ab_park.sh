#!/bin/bash
# Persistent kernel: boundary chunks parked in LDS and stored by the sweep (shipped
# candidate) vs stored by their owner with byte masks (build_variants/nopark), in
# one process on the bimodal batch, twice; then the GPU tests on the new tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/park; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=hysteria_amd/libhyobfs.so; V=build_variants/libhyobfs_nopark.so
for i in 1 2; do
  AB_WORKLOAD=bimodal step ab_bimodal_$i 300 python -u scripts/ab_inproc.py $L:persistent $V:persistent > $O/ab_bimodal_$i.txt 2>&1
done
step pytest 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_one.py bimodal 5
done
echo done
