#!/bin/bash
# Round-2 GPU session steps; each GPU step has its own time limit and the first
# failure ends the script.  Usage: scripts/gpu_r02.sh "ab test bench n2 prof"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
MODE=${1:-"ab test bench"}
for m in $MODE; do
  case $m in
    ab) step ab 300 python -u scripts/ab_kernels.py wave,uniform 1200 > "$OUT/ab_1200.txt" 2>&1
        step ab1192 300 python -u scripts/ab_kernels.py wave,uniform 1192 > "$OUT/ab_1192.txt" 2>&1 ;;
    test) step pytest 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 ;;
    bench) step bench 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    n2) step bench_n2 400 python bench.py --gpus 2 --no-cpu-baseline > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" ;;
    prof) step collect 900 bash scripts/collect_profiles.sh r02 > "$OUT/collect.log" 2>&1 ;;
  esac
done
echo done
