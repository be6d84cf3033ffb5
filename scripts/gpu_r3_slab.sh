#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python scripts/ab_launches.py "wgrad_slab_mb=8" "wgrad_slab_mb=12" "wgrad_slab_mb=16" "wgrad_slab_mb=24" > gpurun_out/ab_slab.txt 2>&1 || { tail -n 20 gpurun_out/ab_slab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_slab.txt
MODEL=rpv TAG=r3_rpv_v3 bash scripts/gpu_pmc.sh > gpurun_out/pmc_rpv_v3_summary.txt 2>&1 || { tail -n 10 gpurun_out/pmc_rpv_v3_summary.txt; exit 1; }
grep -A2 "conv_stack\|dual_halo\|wgrad_halo\|head_kernel\|reduce_optim\|dense_bwd\|prologue\|dense_splitk" gpurun_out/r3_rpv_v3_pmc.txt | grep -- "->\|\[" | head -30
