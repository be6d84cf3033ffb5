#!/bin/bash
# Round-4 pass P: re-check of the launch-geometry defaults at the final kernels (co-scheduled
# dgrad block count / n-tiles, conv-stack row bands, dense dX tiles), then steps per graph.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STEPS=600 bash scripts/ab_tunes.sh "" "dgrad_min_wgs=512" "stack_splits=4" "dgrad_ntc=2" "dx_min_wgs=256" \
  > gpurun_out/r4p_ab_rpv.txt 2>&1 || { cat gpurun_out/r4p_ab_rpv.txt; exit 1; }
cat gpurun_out/r4p_ab_rpv.txt
for i in 1 2; do for g in 8 16 32; do
  r=$(timeout -k 10 120 python bench.py --steps 640 --warmup 64 --no-hpo --steps-per-graph $g 2>/dev/null | tail -n 1) || exit 1
  echo "r$i [spg=$g] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/r4p_spg.txt
