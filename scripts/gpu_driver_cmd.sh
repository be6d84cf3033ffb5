#!/bin/bash
# The round driver's exact 1-GPU command (20 timed steps after 5 warmup, inline HPO on) next
# to a long run: how much the short run's number differs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv$i.log 2>&1 || { tail -n 20 gpurun_out/drv$i.log; exit 1; }
  tail -n 1 gpurun_out/drv$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("driver-cmd", d["ms_per_step"], d["value"], d["config"].get("step_ms_p50"), d["config"].get("step_ms_max"))'
done
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/long.log 2>&1 || exit 1
tail -n 1 gpurun_out/long.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("long", d["ms_per_step"], d["value"])'
