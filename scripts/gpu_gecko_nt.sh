#!/bin/bash
# Gecko encode: nontemporal vs plain stores (alternating processes) + WRITE_SIZE of each
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/gknt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 120 python3 -u $R/scripts/aux_bench.py > $O/aux_nt1_$r.json 2>/dev/null || exit 1
  HYOBFS_LIB=$R/build_variants/libhyobfs_nt0.so timeout -k 10 120 python3 -u $R/scripts/aux_bench.py > $O/aux_nt0_$r.json 2>/dev/null || exit 1
done
echo timed
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_nt1 -o run -- python3 $R/scripts/aux_bench.py > $O/w_nt1.log 2>&1 || exit 1
HYOBFS_LIB=$R/build_variants/libhyobfs_nt0.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_nt0 -o run -- python3 $R/scripts/aux_bench.py > $O/w_nt0.log 2>&1 || exit 1
echo done
