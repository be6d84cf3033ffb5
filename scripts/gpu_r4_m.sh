#!/bin/bash
# Round-4 pass M: first-layer wgrad geometry A/B (split count -> pipelined staging with the
# pooled-dY expansion; 512-pixel blocks).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STEPS=600 bash scripts/ab_tunes.sh "" "wgrad_splits0=256" "wgrad_splits0=400" "wgrad_splits0=480" \
  "wgrad_block_px0=512" "wgrad_block_px0=512,wgrad_splits0=256" "wgrad_block_px0=512,wgrad_splits0=384" \
  > gpurun_out/r4m_ab_rpv.txt 2>&1 || { cat gpurun_out/r4m_ab_rpv.txt; exit 1; }
cat gpurun_out/r4m_ab_rpv.txt
