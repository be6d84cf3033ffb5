#!/bin/bash
# INTML_TUNE sweep of the 1-GPU bench: one INTML_TUNE value per line of $TUNES (a file; the
# word "default" = unset), each run twice in interleaved rounds; prints ms/step per run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/tune_sweep.txt
: > $out
for round in 1 2; do
  while IFS= read -r tv; do
    [ -z "$tv" ] && continue
    t="$tv"; [ "$tv" = default ] && t=""
    INTML_TUNE="$t" timeout -k 10 180 python bench.py --model ${MODEL:-rpv} --steps ${STEPS:-400} --warmup 40 --no-hpo > gpurun_out/tune_one.log 2>&1 || { echo "FAILED: $tv"; tail -n 20 gpurun_out/tune_one.log; exit 1; }
    ms=$(tail -n 1 gpurun_out/tune_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "r$round $ms $tv" | tee -a $out
  done < "$TUNES"
done
