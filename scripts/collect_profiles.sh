#!/bin/bash
# Round evidence on one MI355X: PMC traffic, kernel-trace stats of the bench
# command, and the bench JSON line.  Results in gpurun_out/profiles/; copy the
# ones to keep into profiles/ (named per round).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/profiles; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
# 1. HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$O/pmc_$c" -o run -- \
    python3 "$R/scripts/prof_one.py" uniform 5 > "$O/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 "$R/scripts/pmc_traffic.py" "$O" > "$O/pmc_traffic.json" || exit 1
cp "$O/pmc_traffic.json" "$R/profiles/pmc_traffic.json"   # box copy only: also copy gpurun_out/profiles/pmc_traffic.json into profiles/ here
# 2. kernel trace + stats of the bench command itself
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-parity > "$O/kt_bench.log" 2>&1 || { echo "kt failed"; exit 1; }
# 3. the bench line (default configuration, CPU baseline included)
cd "$R" && timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py --workload bimodal --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_bimodal.json" 2>> "$O/bench.err" || { echo "bench bimodal failed"; exit 1; }
echo collected
