#!/bin/bash
# Round 3: tile kernel launches split into 1M-datagram chunks -- GPU parity with tiny chunks
# (5 tiles) and the default, size probe with the default and with one launch (0).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03aj
mkdir -p $O
HYOBFS_TILE_LAUNCH_TILES=5 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_chunk5.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u scripts/size_probe.py 8 > $O/size_probe_default.txt 2>&1
HYOBFS_TILE_LAUNCH_TILES=0 timeout -k 10 300 python -u scripts/size_probe.py 8 > $O/size_probe_one.txt 2>&1
echo done
