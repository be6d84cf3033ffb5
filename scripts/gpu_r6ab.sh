#!/bin/bash
# round 6: softmax head logits by recursive halving (17 cross-lane moves instead of 96)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6ab AB_MODEL=mnist AB_ROUNDS=2 AB_STEPS=600
export TESTS="tests/test_hip_kernels.py tests/test_hip_model.py -k 'mnist or head or odd'"
export AB="|"
bash scripts/gpu_pass.sh || exit 1
MODEL=mnist timeout -k 10 200 python scripts/head_timeline.py > gpurun_out/r6ab_head_mnist.txt 2>&1 || { tail -n 20 gpurun_out/r6ab_head_mnist.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6ab_head_mnist.txt
MODEL=mnist STEPS=20 WARMUP=5 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6ab_mnist_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_mnist/run_kernel_trace.csv > gpurun_out/r6ab_mnist_sequence.txt
cat gpurun_out/r6ab_mnist_sequence.txt
