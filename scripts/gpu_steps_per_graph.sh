#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/spg.txt
for r in 1 2; do for k in 8 16 32; do
  timeout -k 10 180 python bench.py --steps 512 --warmup 64 --no-hpo --steps-per-graph $k > gpurun_out/spg.log 2>&1 || { tail -n 20 gpurun_out/spg.log; exit 1; }
  echo "r$r spg=$k $(tail -n 1 gpurun_out/spg.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a gpurun_out/spg.txt
done; done
