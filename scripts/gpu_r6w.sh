#!/bin/bash
# round 6: head's split-K dense epilogue with four tasks' partial loads in flight per thread
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6w AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py tests/test_hip_model.py -k 'dense_and_head or head or legacy'"
bash scripts/gpu_pass.sh || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6w_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6w_legacy_sequence.txt
head -4 gpurun_out/r6w_legacy_sequence.txt; tail -1 gpurun_out/r6w_legacy_sequence.txt
MODEL=rpv STEPS=20 WARMUP=5 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6w_rpv_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv/run_kernel_trace.csv > gpurun_out/r6w_rpv_sequence.txt
head -4 gpurun_out/r6w_rpv_sequence.txt; tail -1 gpurun_out/r6w_rpv_sequence.txt
