#!/bin/bash
# Round 3 host-to-host evidence (BASELINE configs[4]) on the final tree: conn/Gecko GPU
# tests, the pinned H2D/kernel/D2H pipeline, loopback UDP in every PacketConn shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03host; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gecko.py -x -v -m gpu --timeout 120 --timeout-method thread -k "conn or gecko or encode or parse or host" > $O/pytest_host.log 2>&1
step host_bench 240 python scripts/host_bench.py 5 > $O/host_bench.json
step udp_raw 60 ./tools/udp_bench raw 4 4 1200 1024 > $O/udp_raw.json
step udp_single 60 ./tools/udp_bench single 4 4 1200 1024 > $O/udp_single.json
step udp_batch 60 ./tools/udp_bench batch 4 4 1200 1024 > $O/udp_batch.json
step udp_batch8 60 ./tools/udp_bench batch 8 4 1200 1024 > $O/udp_batch8.json
step udp_co_4x2 60 ./tools/udp_bench coalesce 4 4 1200 1024 2 50 > $O/udp_co_4x2.json
step udp_co_4x4 60 ./tools/udp_bench coalesce 4 4 1200 1024 4 50 > $O/udp_co_4x4.json
echo done
