#!/bin/bash
# round 6: legacy PMC passes at the current kernels (first-layer conv / wgrad diagnosis)
set -o pipefail
cd $GRAFT_REPO_ROOT
MODEL=rpv_legacy TAG=r6u_legacy bash scripts/gpu_pmc.sh || exit 1
