#!/bin/bash
# The N=1 native-comm worker (tests/comm_worker_gpu.py) under extra INTML_TUNE flags: how far
# the DP step's weights are from the single-GPU step's after 4 steps, per executor variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "" ",pro_free=0,opt_packs=0" ",pro_free=0" ",opt_tiles=0"; do
  sed "s/comm_capture=1\"/comm_capture=1$v\"/; s/comm_capture=0\"/comm_capture=0$v\"/" tests/comm_worker_gpu.py > gpurun_out/cw.py
  PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 240 python gpurun_out/cw.py gpurun_out/cw.json > gpurun_out/cw.log 2>&1 || { echo "variant $v failed"; tail -n 20 gpurun_out/cw.log; exit 1; }
  python -c "
import json; r=json.load(open('gpurun_out/cw.json'))['train']
print('variant [$v]', {k: (r[k]['p999_abs_diff'], r[k]['max_abs_diff']) for k in ('captured','segmented')}, 'cap_vs_seg', r['captured_vs_segmented'])"
done
