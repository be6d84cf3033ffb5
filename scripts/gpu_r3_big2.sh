#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python scripts/ab_launches.py --model legacy --rounds 3 "conv_big=0" "conv_big=1" > gpurun_out/ab_big.txt 2>&1 || { tail -n 20 gpurun_out/ab_big.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_big.txt
INTML_GL5=1 $T 300 python scripts/ab_launches.py --model legacy --rounds 3 "conv_big=1" > gpurun_out/ab_big5.txt 2>&1 || { tail -n 20 gpurun_out/ab_big5.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_big5.txt
