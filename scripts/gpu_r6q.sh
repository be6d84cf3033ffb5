#!/bin/bash
# round 6: halo-staged conv without per-step divisions; 16-wave / 512-row blocks; strided dgrads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6q AB_MODEL=rpv_legacy AB_ROUNDS=3 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k 'legacy or wide' tests/test_dense_bwd.py"
export AB="|conv_hs_wv=16|conv_hs_dil=0|dw_late=1"
bash scripts/gpu_pass.sh || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6q_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6q_legacy_sequence.txt
cat gpurun_out/r6q_legacy_sequence.txt
INTML_TUNE=conv_hs_wv=16 MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6q_legacy_stats_wv16.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6q_legacy_sequence_wv16.txt
cat gpurun_out/r6q_legacy_sequence_wv16.txt
