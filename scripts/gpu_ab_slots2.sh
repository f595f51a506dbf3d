#!/bin/bash
# Bimodal batch: the packed wave kernel's park slots (96 / 128 default / 160) and
# run length (HYOBFS_PACKED_RUN_LOG2 = 6, 4, 3; read once per process), against
# the persistent kernel in the same process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/slots2; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=hysteria_amd/libhyobfs.so
AB_WORKLOAD=bimodal step ab_slots 400 python -u scripts/ab_inproc.py $L:persistent $L:wave build_variants/libhyobfs_slots96.so:wave build_variants/libhyobfs_slots160.so:wave > $O/ab_slots.txt 2>&1
for rl in 4 3; do
  HYOBFS_PACKED_RUN_LOG2=$rl AB_WORKLOAD=bimodal step ab_run$rl 400 python -u scripts/ab_inproc.py $L:persistent $L:wave build_variants/libhyobfs_slots160.so:wave > $O/ab_run$rl.txt 2>&1
done
echo done
