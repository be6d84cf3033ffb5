#!/bin/bash
# round 6: MNIST dual conv2 (41.6 us, the largest kernel of the MNIST step) launch-geometry sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6x AB_MODEL=mnist AB_ROUNDS=2 AB_STEPS=600
export AB="|dgrad_ntc=2|dgrad_min_wgs=512|dgrad_min_wgs=128|wgrad_block_px=128|wgrad_block_px=512|wgrad_max_rows1=4"
bash scripts/gpu_pass.sh || exit 1
