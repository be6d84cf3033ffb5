#!/bin/bash
# wgrad geometry sweep (per-launch A/B): splits cap and rows per block
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 180 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py -x > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 2 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 400 python scripts/ab_launches.py "wgrad_splits=1024" "wgrad_splits=256" "wgrad_splits=384" "wgrad_splits=512" "wgrad_splits=768" "wgrad_block_px0=512" "wgrad_block_px0=128" "wgrad_block_px0=512,wgrad_splits=384" > gpurun_out/sweep_wgrad.txt 2>&1 || { tail -n 20 gpurun_out/sweep_wgrad.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/sweep_wgrad.txt
