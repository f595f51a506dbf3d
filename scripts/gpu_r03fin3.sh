#!/bin/bash
# Round 3 final evidence (after the tile launch split) for the tree as it is: GPU suite, smoke, PMC traffic and
# kernel-trace stats (collect_profiles.sh), the bench line (reading the fresh traffic
# entry), the (f)-row rates and their VALU counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/r03fin3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash scripts/collect_profiles.sh r03fin3 > $O/collect.log 2>&1 || { echo "collect failed"; exit 1; }
cp gpurun_out/profiles/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python -u scripts/aux_bench.py > $O/aux_bench.json 2> $O/aux_bench.err || { echo "aux failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_aux -o run -- python3 $R/scripts/aux_bench.py > $O/pmc_aux.log 2>&1 || { echo "pmc aux failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_aux -o run -- python3 $R/scripts/aux_bench.py > $O/kt_aux.log 2>&1 || { echo "kt aux failed"; exit 1; }
echo done
