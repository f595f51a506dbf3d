#!/bin/bash
# Ablation: wave kernel without its boundary step (wrong output; timing and
# FETCH_SIZE only) against the shipped build.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abw3; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u scripts/ab_inproc.py hysteria_amd/libhyobfs.so:wave build_variants/libhyobfs_nobound.so:wave > $O/ab_uniform.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
HYOBFS_LIB=$R/build_variants/libhyobfs_nobound.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/F_nob -o run -- python3 $R/scripts/prof_one.py uniform 3 wave > $O/F_nob.log 2>&1 || exit 1
echo done
