#!/bin/bash
# Inline-HPO engines per GPU (the `hpo` record of the default bench line): 3 / 4 / 5 / 6.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/hpo_engines.txt
for e in 3 4 5 6; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --hpo-engines-per-gpu $e > gpurun_out/hpoe.log 2>&1 || { tail -n 20 gpurun_out/hpoe.log; exit 1; }
  echo "engines $e $(tail -n 1 gpurun_out/hpoe.log | python -c 'import json,sys; h=json.loads(sys.stdin.read())["hpo"]; print(h["trials_per_hour"], h["wall_s"], h["mean_trial_s"], h["trials_done"])')" | tee -a gpurun_out/hpo_engines.txt
done
