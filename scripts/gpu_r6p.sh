#!/bin/bash
# round 6: halo-staged conv for the strided dgrads (parity classes; 4-tile blocks for the
# 64-channel conv2 dgrad) vs conv_gl's per-tap row gather
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6p AB_MODEL=rpv_legacy AB_ROUNDS=3 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k 'legacy or wide' tests/test_dense_bwd.py"
export AB="|conv_hs_dil=0"
bash scripts/gpu_pass.sh || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6p_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6p_legacy_sequence.txt
cat gpurun_out/r6p_legacy_sequence.txt
