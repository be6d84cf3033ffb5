#!/bin/bash
# round 6: dense wgrad + fused Adam grid order (0: feature groups fastest; 1: n groups of a
# feature group consecutive; 2: same + XCD-contiguous tile ranges) and the gradient store skip
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6n AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export TESTS="tests/test_dense_bwd.py"
export AB="|dw_order=1|dw_order=2|opt_nograd=1|dw_order=2,opt_nograd=1"
bash scripts/gpu_pass.sh || exit 1
INTML_TUNE=dw_order=2 MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6n_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6n_legacy_sequence.txt
cat gpurun_out/r6n_legacy_sequence.txt
