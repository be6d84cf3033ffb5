#!/bin/bash
# Round-4 pass S: dense wgrad n-tiles per workgroup (8 -> 4 / 2: 2x / 4x the workgroups).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROUNDS=2 STEPS=600 bash scripts/ab_tunes.sh "" "dw_ntt=4" "dw_ntt=2" > gpurun_out/r4s_ab_rpv.txt 2>&1 || { cat gpurun_out/r4s_ab_rpv.txt; exit 1; }
cat gpurun_out/r4s_ab_rpv.txt
ROUNDS=2 BENCH_ARGS="--model mnist" bash scripts/ab_tunes.sh "" "dw_ntt=4" "dw_ntt=2" > gpurun_out/r4s_ab_mnist.txt 2>&1 || { cat gpurun_out/r4s_ab_mnist.txt; exit 1; }
cat gpurun_out/r4s_ab_mnist.txt
