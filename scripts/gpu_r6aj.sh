#!/bin/bash
# round 6: halo-staged conv with the n-blocks of a row block on one XCD (adjacent ids, shared L2)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6aj AB_MODEL=rpv_legacy AB_ROUNDS=3 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k 'legacy_conv_variants'"
export AB="|conv_hs_order=1"
bash scripts/gpu_pass.sh || exit 1
INTML_TUNE=conv_hs_order=1 MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6aj_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6aj_legacy_sequence.txt
grep -E "conv_hs|step:" gpurun_out/r6aj_legacy_sequence.txt
