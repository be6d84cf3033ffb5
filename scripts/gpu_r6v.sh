#!/bin/bash
# round 6: legacy first conv (conv_halo, 4-tile blocks): 2 m-tiles per wave per pass (half the
# epilogue staging LDS: 4 instead of 3 workgroups per CU) and smaller row blocks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6v AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k 'legacy_conv_variants'"
export AB="|halo_tm=2|halo_min_wgs=2048|halo_tm=2,halo_min_wgs=2048"
bash scripts/gpu_pass.sh || exit 1
INTML_TUNE=halo_tm=2 MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6v_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6v_legacy_sequence.txt
cat gpurun_out/r6v_legacy_sequence.txt
