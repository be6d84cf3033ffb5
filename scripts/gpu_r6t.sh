#!/bin/bash
# round 6: wide-conv wgrad split count = one residency wave of workgroups (default) vs two
# (wgrad_tile_fill=2) vs the previous 1024-workgroup target
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6t AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k 'legacy or wide'"
export AB="|wgrad_tile_fill=2|wgrad_tile_wgs=1024"
bash scripts/gpu_pass.sh || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6t_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6t_legacy_sequence.txt
cat gpurun_out/r6t_legacy_sequence.txt
