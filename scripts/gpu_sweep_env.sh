#!/bin/bash
# Env-knob sweep of the 1-GPU RPV bench (via gpurun): SWEEP="VAR=a VAR=b ..." (space separated
# assignments, each may hold several comma-joined VAR=val pairs separated by ';').
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/sweep.txt
for cfg in $SWEEP; do
  envs=$(echo "$cfg" | tr ';' ' ')
  timeout -k 10 120 env $envs python bench.py --model ${MODEL:-rpv} --steps 300 --warmup 30 --no-dp-delta > gpurun_out/sweep_one.log 2>&1 || { tail -n 20 gpurun_out/sweep_one.log; exit 1; }
  v=$(tail -n 1 gpurun_out/sweep_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
  echo "$cfg $v" | tee -a gpurun_out/sweep.txt
done
