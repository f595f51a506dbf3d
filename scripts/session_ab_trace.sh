#!/bin/bash
# tests + in-process A/B of variant libraries + kernel trace of the default library
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; tail -1 $O/pytest_gpu.log
grep -E "^FAILED" $O/pytest_gpu.log | head -3
timeout -k 10 300 python scripts/ab_inproc.py hysteria_amd/libhyobfs.so "$@" 2>&1 | grep -v amdgpu.ids
AB_WORKLOAD=bimodal timeout -k 10 300 python scripts/ab_inproc.py hysteria_amd/libhyobfs.so "$@" 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/scripts/prof_one.py uniform 5 > $R/$O/kt.log 2>&1
cut -d, -f1-4 $R/$O/kt/run_kernel_stats.csv | head -8
