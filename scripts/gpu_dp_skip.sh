#!/bin/bash
# Where the data-parallel step's extra time goes at N = 1 (INTML_DP_FORCE=1): the DP bench
# with one launch dropped from the captured step (timing only) vs the non-DP bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/dp_skip.txt
: > $out
timeout -k 10 180 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/dps.log 2>&1 || { tail -n 20 gpurun_out/dps.log; exit 1; }
echo "non-DP $(tail -n 1 gpurun_out/dps.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a $out
for sk in none reduce_b0 allreduce_b0 optim_b0; do
  if [ "$sk" = none ]; then tv=""; else tv="skip=$sk"; fi
  INTML_DP_FORCE=1 INTML_TUNE="$tv" timeout -k 10 180 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/dps.log 2>&1 || { echo "$sk failed"; tail -n 20 gpurun_out/dps.log; exit 1; }
  echo "DP skip=$sk $(tail -n 1 gpurun_out/dps.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a $out
done
