#!/bin/bash
# Round 3: wave-kernel sweep, unconditional loads (main, U=8), software pipelined (pipe U=4,
# pipe6 U=6) against prev (conditional loads) on configs[2] and the uniform batch under
# the wave kernel; wires compared with main's.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ac
mkdir -p $O
L="main=hysteria_amd/libhyobfs.so,prev=build_variants/libhyobfs_prev.so,pipe=build_variants/libhyobfs_pipe.so,pipe6=build_variants/libhyobfs_pipe6.so"
for rep in 1 2; do
  AB_LIBS=$L AB_WORKLOAD=bimodal timeout -k 10 300 python -u scripts/ab_variants.py auto > $O/ab_bimodal_$rep.txt 2>&1
done
AB_LIBS=$L timeout -k 10 300 python -u scripts/ab_variants.py wave > $O/ab_uniform_wave.txt 2>&1
echo done
# Gecko encode: the same pipelining of the aligned sweep (gkpipe U=4 at the 6-wave cap, gkpipe2 U=2,
# gkpipe4w5 U=4 at a 5-wave cap) against main
for rep in 1 2; do
  AB_LIBS="main=hysteria_amd/libhyobfs.so,gkpipe=build_variants/libhyobfs_gkpipe.so,gkpipe2=build_variants/libhyobfs_gkpipe2.so,gkpipe4w5=build_variants/libhyobfs_gkpipe4w5.so" \
    timeout -k 10 300 python -u scripts/ab_gecko_variants.py > $O/ab_gecko_$rep.txt 2>&1
done
echo done-gecko
