#!/bin/bash
# round 6: 3-slot LDS ring for the big LDS-DMA conv blocks (conv_gl<8,8>: 72 KB, two blocks per
# CU) vs the 4-slot default, on the legacy model and on the bench model
set -o pipefail
cd $GRAFT_REPO_ROOT
export AB_ROUNDS=3 AB_STEPS=150
TAG=r6m_legacy AB_MODEL=rpv_legacy AB="|conv_gl_nbuf=3" bash scripts/gpu_pass.sh || exit 1
TAG=r6m_rpv AB_MODEL=rpv AB_STEPS=600 AB="|conv_gl_nbuf=3" bash scripts/gpu_pass.sh || exit 1
