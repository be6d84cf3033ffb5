#!/bin/bash
# round 6: slab partials per reduction lane on the RPV / MNIST steps (8 and 4 measured worse in round 5)
set -o pipefail
cd $GRAFT_REPO_ROOT
export AB_ROUNDS=2 AB_STEPS=600
TAG=r6ai_rpv AB_MODEL=rpv AB="|red_lanes=32|red_lanes=64" bash scripts/gpu_pass.sh || exit 1
TAG=r6ai_mnist AB_MODEL=mnist AB="|red_lanes=32|red_lanes=64" bash scripts/gpu_pass.sh || exit 1
