#!/bin/bash
# round 6: legacy end-of-step reduction (96 MB of wgrad slabs, 35 us): slab partials per lane;
# dense wgrad + Adam in 2-tile workgroups (74 VGPRs, five workgroups per CU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6z AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export TESTS="tests/test_dense_bwd.py"
export AB="|dw_ntt=8|red_lanes=32"
bash scripts/gpu_pass.sh || exit 1
INTML_TUNE=dw_ntt=8 MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6z_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6z_legacy_sequence.txt
grep -E "dense|reduce|step:" gpurun_out/r6z_legacy_sequence.txt
