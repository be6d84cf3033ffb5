#!/bin/bash
# round 6: RPV B=1024 launch-geometry sweep (defaults were tuned at B=128)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6ah AB_MODEL=rpv AB_ROUNDS=2 AB_STEPS=100 AB_ARGS="--batch 1024"
export AB="|wgrad_block_px=512|wgrad_block_px0=1024|dgrad_min_wgs=512|dgrad_ntc=2|wgrad_max_rows=16|red_lanes=32"
bash scripts/gpu_pass.sh || exit 1
