#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python scripts/ab_launches.py "pro_dbg=0" "pro_dbg=1" "pro_dbg=2" > gpurun_out/ab_pro.txt 2>&1 || { tail -n 20 gpurun_out/ab_pro.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_pro.txt | head -3
$T 200 python scripts/head_timeline.py > gpurun_out/head_timeline.txt 2>&1 || { tail -n 20 gpurun_out/head_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/head_timeline.txt | tail -n 25
$T 200 python scripts/bwd_timeline.py > gpurun_out/bwd_timeline.txt 2>&1 || { tail -n 20 gpurun_out/bwd_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bwd_timeline.txt | tail -n 25
