#!/bin/bash
# round 6: legacy conv4 forward (conv_gl<8,4,4>, 256 x 2 blocks) on the big 8-wave blocks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6af AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export AB="|conv_big_min=256|conv_big_min=128"
bash scripts/gpu_pass.sh || exit 1
