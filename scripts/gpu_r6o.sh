#!/bin/bash
# round 6: legacy dense dX epilogue through LDS (16-byte runs); dense wgrad grid order and the
# gradient store skip re-measured over 3 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6o AB_MODEL=rpv_legacy AB_ROUNDS=3 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k dense_and_head tests/test_dense_bwd.py"
export AB="|dw_order=1|opt_nograd=1|dw_order=1,opt_nograd=1"
bash scripts/gpu_pass.sh || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6o_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6o_legacy_sequence.txt
cat gpurun_out/r6o_legacy_sequence.txt
