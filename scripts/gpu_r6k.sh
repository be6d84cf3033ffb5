#!/bin/bash
# round 6: halo-staged wide conv (conv_hs_kernel) -- kernel numerics (forward / dgrad / wgrad of
# every legacy and wide test layer vs fp32 PyTorch), legacy A/B against the LDS-DMA gather
# (INTML_TUNE=conv_hs=0), per-launch sequence of the legacy step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TESTS="tests/test_hip_kernels.py tests/test_hip_model.py" TAG=r6k AB_MODEL=rpv_legacy AB_ROUNDS=3 AB_STEPS=150
export AB="|conv_hs=0"
bash scripts/gpu_pass.sh || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6k_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6k_legacy_sequence.txt
cat gpurun_out/r6k_legacy_sequence.txt
