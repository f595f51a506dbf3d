#!/bin/bash
# Round 3: Gecko keyed padding on the GPU (tests, rate) and counter rooflines of the
# compute-bound (f) kernels (Gecko encode, realm punch matcher, QUIC open).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/r03g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gecko.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gecko.log 2>&1
timeout -k 10 300 python -u scripts/aux_bench.py > $O/aux_bench.json 2> $O/aux_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_aux -o run -- python3 $R/scripts/aux_bench.py > $O/kt_aux.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_aux -o run -- python3 $R/scripts/aux_bench.py > $O/pmc_aux.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_quic -o run -- python3 $R/scripts/bench_quic.py --n 65536 --steps 3 --warmup 1 --no-cpu > $O/pmc_quic.log 2>&1
echo done
