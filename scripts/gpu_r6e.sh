#!/bin/bash
# round 6: B=1024 launch-geometry A/B (conv-stack row bands: the specialised RPV stack instance
# needs >= 2 bands; at B=1024 the default picks 1 and runs the generic kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6e AB_ROUNDS=2 AB_STEPS=400 AB_ARGS="--batch 1024"
export AB="|stack_splits=2|stack_splits=4|stack_splits=2,stack_spec=1"
bash scripts/gpu_pass.sh
