#!/bin/bash
# Persistent kernel: boundary chunks per sweep window vs once per sub-tile
# (bimodal, one process) + FETCH/WRITE of the shipped build on bimodal.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abb2; mkdir -p $O
cd $R
AB_WORKLOAD=bimodal timeout -k 10 300 python3 -u scripts/ab_inproc.py hysteria_amd/libhyobfs.so build_variants/libhyobfs_prev.so hysteria_amd/libhyobfs.so > $O/ab_bimodal.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/ab_inproc.py hysteria_amd/libhyobfs.so:persistent build_variants/libhyobfs_prev.so:persistent > $O/ab_uniform_persistent.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- python3 $R/scripts/prof_one.py bimodal 3 > $O/$c.log 2>&1 || exit 1
done
echo done
