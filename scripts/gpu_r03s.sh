#!/bin/bash
# Round 3: kernel-trace stats of the packed scan launches (main vs prev) on configs[2].
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/main -o run -- python3 scripts/prof_one.py bimodal 10 > $O/main.log 2>&1
HYOBFS_LIB=build_variants/libhyobfs_prev.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prev -o run -- python3 scripts/prof_one.py bimodal 10 > $O/prev.log 2>&1
echo done
