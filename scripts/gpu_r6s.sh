#!/bin/bash
# round 6: legacy wide-conv wgrad split counts -- slab budgets around 32 MB, and per-kernel
# sequences of the 32 MB budget vs the 512-workgroup target (similar split counts, 10 % apart)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6s AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export AB="wgrad_tile_slab_mb=32|wgrad_tile_slab_mb=24|wgrad_tile_slab_mb=40|wgrad_tile_slab_mb=48|wgrad_tile_slab_mb=32,wgrad_tile_wgs=2048"
bash scripts/gpu_pass.sh || exit 1
for t in wgrad_tile_slab_mb=32 wgrad_tile_wgs=512; do
  INTML_TUNE=$t MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6s_stats_$t.txt || exit 1
  python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6s_sequence_$t.txt
  cat gpurun_out/r6s_sequence_$t.txt
done
