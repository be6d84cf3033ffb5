#!/bin/bash
# Round-4 pass O: split count of the dual launches' wgrad (the slab budget caps RPV conv2 at
# 86 splits of 3 blocks; its wgrad is the dual conv2 launch's long pole) and conv2 row blocks.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STEPS=600 bash scripts/ab_tunes.sh "" "wgrad_slab_mb=16" "wgrad_slab_mb=32" "wgrad_block_px2=64" \
  > gpurun_out/r4o_ab_rpv.txt 2>&1 || { cat gpurun_out/r4o_ab_rpv.txt; exit 1; }
cat gpurun_out/r4o_ab_rpv.txt
ROUNDS=2 BENCH_ARGS="--model mnist" bash scripts/ab_tunes.sh "" "wgrad_slab_mb=16" "wgrad_slab_mb=32" \
  > gpurun_out/r4o_ab_mnist.txt 2>&1 || { cat gpurun_out/r4o_ab_mnist.txt; exit 1; }
cat gpurun_out/r4o_ab_mnist.txt
