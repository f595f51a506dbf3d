#!/bin/bash
# Host-to-host measurements (BASELINE configs[4], DESIGN.md "Host-to-host"):
# the pinned H2D/kernel/D2H pipeline and the loopback-UDP PacketConn wrapper.
# Every step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/host; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@"; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step host_bench 240 python scripts/host_bench.py 5 > $O/host_bench.json
for m in raw batch single; do
  step "udp_$m" 60 ./tools/udp_bench $m 4 4 1200 1024 > $O/udp_$m.json
done
step udp_batch_8 60 ./tools/udp_bench batch 8 4 1200 1024 > $O/udp_batch8.json
nproc > $O/nproc.txt
echo done
