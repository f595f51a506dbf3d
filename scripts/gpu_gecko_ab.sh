#!/bin/bash
# Gecko encode: GPU tests, aligned sweep vs plaintext windows (alternating
# processes), then counter passes on the shipped library.
set -u
O=gpurun_out/gk; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest 300 python -u -m pytest tests/test_gpu_gecko.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for r in 1 2; do
  step aligned$r 120 python -u scripts/aux_bench.py > $O/aux_aligned$r.json 2> $O/aux_aligned$r.err
  HYOBFS_LIB=build_variants/libhyobfs_gkwin.so step windows$r 120 python -u scripts/aux_bench.py > $O/aux_windows$r.json 2> $O/aux_windows$r.err
done
step pmc 600 bash scripts/pmc_gecko.sh > $O/pmc.log 2>&1
echo done
