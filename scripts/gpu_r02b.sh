#!/bin/bash
# Round-2 second session: GPU tests, bench (bimodal after the tile-sum scan
# rewrite), source-keyed profiles, then the coalescing loopback rates with
# latency.  Each GPU step has its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O/host
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
MODE=${1:-"test bench prof udp"}
for m in $MODE; do
  case $m in
    test) step pytest 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 ;;
    quic) step pytest_quic 300 python -u -m pytest tests/test_gpu_quic.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_quic.log 2>&1 ;;
    qbench) step bench_quic 300 python -u scripts/bench_quic.py > $O/bench_quic.json 2> $O/bench_quic.err ;;
    qprof) step qprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/qprof -o run -- python scripts/bench_quic.py --steps 10 > $O/qprof.log 2>&1 ;;
    bench) step bench 300 python bench.py > $O/bench.json 2> $O/bench.err ;;
    prof) step collect 900 bash scripts/collect_profiles.sh r02 > $O/collect.log 2>&1 ;;
    udp)
      step udp_batch 60 ./tools/udp_bench batch 4 4 1200 1024 > $O/host/udp_batch.json
      step udp_co_4x2 60 ./tools/udp_bench coalesce 4 4 1200 1024 2 50 > $O/host/udp_co_4x2.json
      step udp_co_4x4 60 ./tools/udp_bench coalesce 4 4 1200 1024 4 50 > $O/host/udp_co_4x4.json
      step udp_co_1x8 60 ./tools/udp_bench coalesce 1 4 1200 1024 8 50 > $O/host/udp_co_1x8.json
      step udp_co_4x2_w20 60 ./tools/udp_bench coalesce 4 4 1200 1024 2 20 > $O/host/udp_co_4x2_w20.json
      step udp_co_4x2_b256 60 ./tools/udp_bench coalesce 4 4 1200 256 2 50 > $O/host/udp_co_4x2_b256.json ;;
  esac
done
echo done
