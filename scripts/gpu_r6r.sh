#!/bin/bash
# round 6: legacy wide-conv wgrad split-K geometry (slab byte budget / workgroup target) -- the
# slabs are what the end-of-step reduction reads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6r AB_MODEL=rpv_legacy AB_ROUNDS=2 AB_STEPS=150
export AB="|wgrad_tile_slab_mb=32|wgrad_tile_slab_mb=16|wgrad_tile_wgs=512|wgrad_tile_wgs=2048"
bash scripts/gpu_pass.sh || exit 1
