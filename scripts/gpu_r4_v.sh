#!/bin/bash
# Round-4 pass V: rocprofv3 kernel stats of the RPV / MNIST / legacy bench steps at the final defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/r4v_rpv_stats.txt || exit 1
head -14 gpurun_out/r4v_rpv_stats.txt
MODEL=mnist bash scripts/prof_model.sh > gpurun_out/r4v_mnist_stats.txt || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 bash scripts/prof_model.sh > gpurun_out/r4v_legacy_stats.txt || exit 1
head -14 gpurun_out/r4v_legacy_stats.txt
