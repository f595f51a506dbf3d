#!/bin/bash
# Round 3: tile kernels with a separate edge step (Gecko encode, packed Salamander) -- GPU parity,
# in-process Salamander A/B, Gecko tile vs wave-group kernel, bench line.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/aux_bench.py > $O/aux_tile_$rep.json 2> $O/aux_tile_$rep.err
  HYOBFS_GECKO_KERNEL=wave timeout -k 10 300 python -u scripts/aux_bench.py > $O/aux_wave_$rep.json 2> $O/aux_wave_$rep.err
done
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so" AB_WORKLOAD=bimodal \
    timeout -k 10 300 python -u scripts/ab_variants.py auto,wave > $O/ab_bimodal_$rep.txt 2>&1
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo done
