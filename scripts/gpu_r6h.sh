#!/bin/bash
# round 6: wgrad row-divisor k-step bases (Wo | 32) -- kernel numerics + A/B against the per-step
# FastDiv path in the same build (INTML_TUNE=wgrad_rowdiv=0), RPV and MNIST
set -o pipefail
cd $GRAFT_REPO_ROOT
export TESTS="tests/test_hip_kernels.py tests/test_hip_model.py" TAG=r6h AB_ROUNDS=3 AB_STEPS=600
export AB="|wgrad_rowdiv=0"
bash scripts/gpu_pass.sh || exit 1
TESTS= TAG=r6h_mnist AB_MODEL=mnist AB_ROUNDS=2 AB="|wgrad_rowdiv=0" bash scripts/gpu_pass.sh
