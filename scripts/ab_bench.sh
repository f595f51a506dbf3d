#!/bin/bash
# A/B the default library against variants in build_variants/, interleaved,
# bench only (no CPU baseline).  Usage: scripts/ab_bench.sh [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
ROUNDS=${1:-2}
for r in $(seq 1 $ROUNDS); do
  for lib in hysteria_amd/libhyobfs.so build_variants/*.so; do
    for wl in ${WLS:-uniform bimodal}; do
      res=$(HYOBFS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>>$OUT/ab.err) || { echo "FAIL $lib $wl"; exit 1; }
      python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('$r', '$(basename $lib)', '$wl', 'obf_ms', round(d['roofline']['avg_launch_ms'],4), 'obf_GBs', d['roofline']['achieved'], 'deobf_GBs', d['deobfuscate']['achieved_GBs'])" "$res"
    done
  done
done
