#!/bin/bash
# Round 3 evidence for the tree as it is: GPU tests, smoke, PMC traffic + kernel trace, bench line.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=${1:-r03a}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
bash scripts/collect_profiles.sh $TAG > $O/collect.log 2>&1
echo done
