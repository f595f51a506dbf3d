#!/bin/bash
# rocprofv3 counter passes (one counter group per pass; no tracing domains
# besides kernel-trace) on scripts/aux_bench.py (Gecko encode/parse, realm punch).  Output under gpurun_out/pmc_gecko/.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/${PMC_OUT:-pmc_gecko}; mkdir -p "$OUT"   # PMC_OUT, HYOBFS_LIB: A/B builds
cd /tmp && export TMPDIR=/tmp
WL=${1:-uniform}
i=0
PASSES=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
[ "${PMC_TRAFFIC_ONLY:-0}" = 1 ] && PASSES=("FETCH_SIZE" "WRITE_SIZE")
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/scripts/aux_bench.py" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done
