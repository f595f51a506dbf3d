#!/bin/bash
# Gecko encode: nontemporal vs plain stores (alternating processes) + WRITE_SIZE of each
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/gknt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 120 python3 -u $R/scripts/aux_bench.py > $O/aux_new_$r.json 2>/dev/null || exit 1
  HYOBFS_LIB=$R/build_variants/libhyobfs_prev.so timeout -k 10 120 python3 -u $R/scripts/aux_bench.py > $O/aux_prev_$r.json 2>/dev/null || exit 1
done
echo timed
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_new -o run -- python3 $R/scripts/aux_bench.py > $O/w_new.log 2>&1 || exit 1
HYOBFS_LIB=$R/build_variants/libhyobfs_prev.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_prev -o run -- python3 $R/scripts/aux_bench.py > $O/w_prev.log 2>&1 || exit 1
echo done
