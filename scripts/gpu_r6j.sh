#!/bin/bash
# round 6: legacy wide-conv staging path A/B -- LDS-DMA gather (conv_gl, default) vs the
# register-staged tile kernel (conv_glds=0) vs 128-row DMA blocks (conv_big=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6j AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export AB="|conv_glds=0|conv_big=0"
bash scripts/gpu_pass.sh || exit 1
INTML_TUNE=conv_glds=0 MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6j_legacy_glds0_stats.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6j_legacy_glds0_sequence.txt
cat gpurun_out/r6j_legacy_glds0_sequence.txt
