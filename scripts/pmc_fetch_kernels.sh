#!/bin/bash
# FETCH_SIZE per kernel variant on the uniform batch, plus a torch copy of the
# same input bytes as the counter's calibration (one pass each).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_fk; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in wave uniform stream persistent; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/$k -o run -- python3 $R/scripts/prof_one.py uniform 3 $k > $O/$k.log 2>&1 || { echo "$k failed"; exit 1; }
  echo "$k ok"
done
cat > /tmp/tcopy.py <<'PY'
import torch
a = torch.empty(1 << 20, 1200, dtype=torch.uint8, device="cuda:0"); a.fill_(7)
b = torch.empty_like(a)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
PY
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/tcopy -o run -- python3 /tmp/tcopy.py > $O/tcopy.log 2>&1 || { echo "tcopy failed"; exit 1; }
echo done
