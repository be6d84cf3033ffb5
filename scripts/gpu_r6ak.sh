#!/bin/bash
# round 6: wide-conv wgrad with the (k, n) tiles of one pixel split adjacent on one XCD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6ak AB_MODEL=rpv_legacy AB_ROUNDS=3 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k 'legacy_conv_variants or wide'"
export AB="|wgrad_tile_order=1"
bash scripts/gpu_pass.sh || exit 1
INTML_TUNE=wgrad_tile_order=1 MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6ak_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6ak_legacy_sequence.txt
grep -E "wgrad_gl|step:" gpurun_out/r6ak_legacy_sequence.txt
