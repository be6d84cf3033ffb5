#!/bin/bash
# Marginal in-graph cost of each launch of the RPV step: the bench with that launch dropped
# from the captured step (INTML_TUNE=skip=..., timing only: results are wrong).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/skip_ablation.txt
: > $out
for sk in none prologue conv_stack_fwd dense_fwd0 head dense_bwd0 wgrad_dgrad_conv2 wgrad_dgrad_conv1 wgrad_conv0 reduce_b0 ${EXTRA_SKIPS}; do
  if [ "$sk" = none ]; then tv=""; else tv="skip=$sk"; fi
  INTML_TUNE="$tv" timeout -k 10 180 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/skip_$sk.log 2>&1 || { echo "$sk failed"; tail -n 20 gpurun_out/skip_$sk.log; exit 1; }
  ms=$(tail -n 1 gpurun_out/skip_$sk.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
  echo "$sk $ms" | tee -a $out
done
