#!/bin/bash
# Wave kernel: nontemporal vs plain input loads, one process, plus FETCH_SIZE of each.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abw2; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u scripts/ab_inproc.py hysteria_amd/libhyobfs.so:wave build_variants/libhyobfs_ntl0.so:wave build_variants/libhyobfs_prev.so:wave > $O/ab_uniform.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/F_nt -o run -- python3 $R/scripts/prof_one.py uniform 3 wave > $O/F_nt.log 2>&1 || exit 1
HYOBFS_LIB=$R/build_variants/libhyobfs_ntl0.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/F_plain -o run -- python3 $R/scripts/prof_one.py uniform 3 wave > $O/F_plain.log 2>&1 || exit 1
echo done
