#!/bin/bash
# Bimodal batch (configs[2]): persistent kernel (default for packed) vs the wave
# kernel with 64 / 128 / 192 park slots per group (HY_PACKED_PARK_SLOTS), one
# process, wire identical across variants; two processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/slots; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=hysteria_amd/libhyobfs.so
for i in 1 2; do
  AB_WORKLOAD=bimodal step ab_$i 400 python -u scripts/ab_inproc.py $L:persistent $L:wave build_variants/libhyobfs_slots128.so:wave build_variants/libhyobfs_slots192.so:wave > $O/ab_$i.txt 2>&1
done
echo done
