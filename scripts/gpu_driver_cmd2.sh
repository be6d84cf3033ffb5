#!/bin/bash
# The driver's short run (20 timed steps after 5 warmup) with and without the inline-HPO engine
# processes alive: does the farm's presence cost the timed steps?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for extra in "--no-hpo" ""; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $extra > gpurun_out/drv.log 2>&1 || { tail -n 20 gpurun_out/drv.log; exit 1; }
    tail -n 1 gpurun_out/drv.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("short ['"$extra"']", d["ms_per_step"], d["config"].get("step_ms_p50"), d["config"].get("step_ms_max"))'
  done
done
