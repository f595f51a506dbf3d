#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/park2; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=hysteria_amd/libhyobfs.so; V=build_variants/libhyobfs_nopark.so
for i in 1 2; do
  AB_WORKLOAD=bimodal step ab_bimodal_$i 300 python -u scripts/ab_inproc.py $L:persistent $V:persistent > $O/ab_bimodal_$i.txt 2>&1
done
cd /tmp && export TMPDIR=/tmp
step pmc_WRITE_SIZE 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_WRITE_SIZE -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_one.py bimodal 5
echo done
