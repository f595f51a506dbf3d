#!/bin/bash
# Evidence for the tree as it is: smoke, GPU tests, source-keyed PMC traffic and
# kernel stats (collect_profiles.sh), then the bench line reading that traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out; mkdir -p $O
TAG=${1:-r02c}
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step pytest 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
step collect 900 bash scripts/collect_profiles.sh $TAG > $O/collect.log 2>&1
cp $O/profiles/pmc_traffic.json profiles/pmc_traffic.json
step bench 300 python bench.py > $O/bench.out 2> $O/bench.err && grep "^{" $O/bench.out > $O/bench.json
echo done
