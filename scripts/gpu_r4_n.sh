#!/bin/bash
# Round-4 pass N: first-layer wgrad blocks of 512 pixels as the default (RPV: 8 rows), against
# the old 256, one-block splits and 16-row blocks; legacy / MNIST unchanged?; the model GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
STEPS=600 bash scripts/ab_tunes.sh "" "wgrad_block_px0=256" "wgrad_splits0=1024" \
  "wgrad_max_rows0=16,wgrad_fit0=0,wgrad_block_px0=1024" > gpurun_out/r4n_ab_rpv.txt 2>&1 || { cat gpurun_out/r4n_ab_rpv.txt; exit 1; }
cat gpurun_out/r4n_ab_rpv.txt
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "wgrad_block_px0=256" \
  > gpurun_out/r4n_ab_legacy.txt 2>&1 || { cat gpurun_out/r4n_ab_legacy.txt; exit 1; }
cat gpurun_out/r4n_ab_legacy.txt
ROUNDS=2 BENCH_ARGS="--model mnist" bash scripts/ab_tunes.sh "" "wgrad_block_px0=256" \
  > gpurun_out/r4n_ab_mnist.txt 2>&1 || { cat gpurun_out/r4n_ab_mnist.txt; exit 1; }
cat gpurun_out/r4n_ab_mnist.txt
$T 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_model.py -m gpu > gpurun_out/r4n_model_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4n_model_tests.log; exit $rc
