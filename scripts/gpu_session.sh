#!/bin/bash
# One GPU-box session: calibration, parity tests, bench, kernel-trace profile.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
MODE=${1:-all}
if [[ $MODE == *calib* || $MODE == all ]]; then
  step calib 180 ./tools/hbm_copy > "$OUT/hbm_copy.json"
fi
if [[ $MODE == *test* || $MODE == all ]]; then
  step pytest 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
if [[ $MODE == *bench* || $MODE == all ]]; then
  step bench 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > "$OUT/bench.json" 2> "$OUT/bench.err"
  step bench_bimodal 300 python bench.py --workload bimodal --steps 10 --warmup 3 --no-cpu-baseline --no-parity > "$OUT/bench_bimodal.json" 2> "$OUT/bench_bimodal.err"
fi
if [[ $MODE == *prof* || $MODE == all ]]; then
  cd /tmp && export TMPDIR=/tmp
  step rocprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-parity > "$OUT/prof_bench.log" 2>&1
fi
echo done
