#!/bin/bash
# Round-4 pass U: geometry re-check after the dense tile changes (co-scheduled dgrad blocks,
# dense dX / wgrad tiles).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROUNDS=2 STEPS=600 bash scripts/ab_tunes.sh "" "dgrad_min_wgs=128" "dx_min_wgs=128" "dw_ntt=2" > gpurun_out/r4u_ab_rpv.txt 2>&1 || { cat gpurun_out/r4u_ab_rpv.txt; exit 1; }
cat gpurun_out/r4u_ab_rpv.txt
