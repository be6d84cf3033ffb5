#!/bin/bash
# round 6: wide-conv wgrad LDS-DMA ring (one 32-pixel k-step per slot, counted waits) vs the
# two-buffer loop (vmcnt(0) at every stage)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6y AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export TESTS="tests/test_hip_kernels.py -k 'legacy_conv_variants or wide'"
export AB="|wgrad_ring=3|wgrad_ring=4"
bash scripts/gpu_pass.sh || exit 1
for t in 3 4; do
INTML_TUNE=wgrad_ring=$t MODEL=rpv_legacy STEPS=10 WARMUP=3 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6y_legacy_stats$t.txt || exit 1
python scripts/prof_sequence.py gpurun_out/prof_rpv_legacy/run_kernel_trace.csv > gpurun_out/r6y_legacy_sequence$t.txt
grep -E "wgrad_g|reduce|step:" gpurun_out/r6y_legacy_sequence$t.txt
done
