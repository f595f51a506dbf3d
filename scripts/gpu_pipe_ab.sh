#!/bin/bash
# Side-lane pipeline (HYOBFS_KERNEL_PIPE) against the wave and in-grid stream
# kernels, one process per schedule, plus a kernel trace of the pipe schedule.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pipe; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step ab_default 240 python -u scripts/ab_kernels.py wave,stream,pipe > $O/ab_default.txt 2>&1
HYOBFS_PIPE_KEY_BLOCKS=1024 step ab_kb1024 240 python -u scripts/ab_kernels.py wave,pipe > $O/ab_kb1024.txt 2>&1
HYOBFS_PIPE_KEY_BLOCKS=64 step ab_kb64 240 python -u scripts/ab_kernels.py wave,pipe > $O/ab_kb64.txt 2>&1
HYOBFS_PIPE_FIRST_RUNS=8192 HYOBFS_PIPE_GROW=8 step ab_f8192_g8 240 python -u scripts/ab_kernels.py wave,pipe > $O/ab_f8192_g8.txt 2>&1
HYOBFS_PIPE_FIRST_RUNS=512 HYOBFS_PIPE_GROW=3 step ab_f512_g3 240 python -u scripts/ab_kernels.py wave,pipe > $O/ab_f512_g3.txt 2>&1
cd /tmp && export TMPDIR=/tmp
AB_ROUNDS=1 AB_STEPS=3 step trace 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_kernels.py pipe > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
echo done
