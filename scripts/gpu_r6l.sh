#!/bin/bash
# round 6: halo-staged conv n-tiles per block for the legacy conv3 forward (8: two blocks per CU,
# default, vs 16) against the LDS-DMA gather (conv_hs=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6l AB_MODEL=rpv_legacy AB_ROUNDS=3 AB_STEPS=150
export AB="|conv_hs_ntc=16|conv_hs=0"
bash scripts/gpu_pass.sh || exit 1
MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6l_legacy_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6l_legacy_sequence.txt
cat gpurun_out/r6l_legacy_sequence.txt
