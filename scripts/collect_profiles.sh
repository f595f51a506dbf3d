#!/bin/bash
# Round evidence on one MI355X for the tree as it is: PMC traffic (uniform and
# bimodal, both directions), kernel-trace stats of the bench command, and the
# bench JSON line.  Results in gpurun_out/profiles/; copy the ones to keep into
# profiles/ (named per round) -- gpurun_out/profiles/pmc_traffic.json is the
# merged traffic file bench.py reads (keyed by the kernel-source hash).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/profiles; mkdir -p "$O"
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp
cp "$R/profiles/pmc_traffic.json" "$O/pmc_traffic.json" 2>/dev/null || echo '{"entries": []}' > "$O/pmc_traffic.json"
# 1. HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes, per workload
for wl in uniform bimodal uniform8m; do   # uniform8m: the N > 1 shard (bench.py at --gpus > 1)
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$O/$wl/pmc_$c" -o run -- \
      python3 "$R/scripts/prof_one.py" $wl 5 > "$O/$wl.pmc_$c.log" 2>&1 || { echo "pmc $wl $c failed"; exit 1; }
  done
  python3 "$R/scripts/pmc_traffic.py" "$O/$wl" $wl "$O/pmc_traffic.json" "$O/pmc_traffic.json" \
    "profiles/${TAG}_pmc/${wl}_{FETCH,WRITE}_SIZE.csv" > "$O/pmc_$wl.txt" || { echo "pmc_traffic $wl failed"; exit 1; }
done
# 2. kernel trace + stats of the bench command itself
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-parity > "$O/kt_bench.log" 2>&1 || { echo "kt failed"; exit 1; }
echo collected
