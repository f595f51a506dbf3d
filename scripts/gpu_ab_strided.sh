#!/bin/bash
# Persistent kernel on the bimodal batch (configs[2]): contiguous per-workgroup
# parts vs interleaved tiles (HYOBFS_PERSIST_ORDER=strided), two processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/strided; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=hysteria_amd/libhyobfs.so
for i in 1 2; do
  AB_WORKLOAD=bimodal step ab_bimodal_$i 300 python -u scripts/ab_inproc.py $L:persistent $L:persistent:HYOBFS_PERSIST_ORDER=strided > $O/ab_bimodal_$i.txt 2>&1
done
step ab_uniform 300 python -u scripts/ab_inproc.py $L:wave $L:persistent $L:persistent:HYOBFS_PERSIST_ORDER=strided > $O/ab_uniform.txt 2>&1
echo done
