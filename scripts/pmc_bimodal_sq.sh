#!/bin/bash
# Counter passes on the configs[2] batch as bench.py runs it (contiguous input, the
# kernel AUTO picks -- the flat kernel since round 6 -- or the one named by $1;
# scripts/prof_one.py bimodal), one counter group per rocprofv3 pass (<= 8 SQ, <= 4 TCC
# counters each).  Results in gpurun_out/pmc_bsq${2:-}/pN/.
set -u
R=$GRAFT_REPO_ROOT
KERN=${1:-auto}
O=$R/gpurun_out/pmc_bsq${2:-}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- \
    python3 $R/scripts/prof_one.py bimodal 3 $KERN > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
