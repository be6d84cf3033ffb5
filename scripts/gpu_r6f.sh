#!/bin/bash
# round 6: the driver's exact 20-step command, host wait policy A/B (ROC_ACTIVE_WAIT_TIMEOUT: how
# long the HIP runtime spins on a completion signal before sleeping on an interrupt).  The GPU
# work is identical; only how fast torch.cuda.synchronize() returns after the last step differs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r6f_wait_ab.txt
: > $O
for i in 1 2 3; do
  for v in "" "ROC_ACTIVE_WAIT_TIMEOUT=5000" "ROC_ACTIVE_WAIT_TIMEOUT=50000"; do
    env $v timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-hpo > gpurun_out/r6f.tmp 2>&1 || { tail -n 20 gpurun_out/r6f.tmp; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/r6f.tmp').read().strip().splitlines()[-1]); print('r$i', '[${v:-default}]', d['value'], d['ms_per_step'], d['config']['step_ms_p50'])" | tee -a $O
  done
done
