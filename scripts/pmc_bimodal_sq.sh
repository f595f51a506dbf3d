#!/bin/bash
# SQ counter passes on the bimodal batch (persistent kernel), one group per pass.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_bsq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  AB_WORKLOAD=bimodal AB_ROUNDS=1 AB_STEPS=3 timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/scripts/ab_inproc.py $R/hysteria_amd/libhyobfs.so:persistent > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
