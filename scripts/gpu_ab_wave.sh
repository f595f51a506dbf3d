#!/bin/bash
# Wave kernel: shipped vs previous build, in one process (uniform and bimodal),
# then FETCH_SIZE / WRITE_SIZE of the shipped build on the uniform batch.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abw; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u scripts/ab_inproc.py hysteria_amd/libhyobfs.so:wave build_variants/libhyobfs_prev.so:wave > $O/ab_uniform.txt 2>&1 || exit 1
AB_WORKLOAD=bimodal timeout -k 10 300 python3 -u scripts/ab_inproc.py hysteria_amd/libhyobfs.so build_variants/libhyobfs_prev.so > $O/ab_bimodal.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- python3 $R/scripts/prof_one.py uniform 3 wave > $O/$c.log 2>&1 || exit 1
done
echo done
