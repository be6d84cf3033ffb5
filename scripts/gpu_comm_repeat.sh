#!/bin/bash
# tests/comm_worker_gpu.py three times (default executor): run-to-run spread of the DP-vs-
# single-GPU weight distance.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 240 python tests/comm_worker_gpu.py gpurun_out/cw$i.json > gpurun_out/cw$i.log 2>&1 || { echo "run $i failed"; tail -n 20 gpurun_out/cw$i.log; exit 1; }
  python -c "
import json; r=json.load(open('gpurun_out/cw$i.json'))['train']
print('run $i', {k: (r[k]['p999_abs_diff'], r[k]['max_abs_diff']) for k in ('captured','segmented')}, 'xgmi', r.get('xgmi', {}).get('p999_abs_diff'))"
done
