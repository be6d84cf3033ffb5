#!/bin/bash
# Round-4 pass A2: A/Bs of the new step variants (RPV, legacy) and the profiling pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STEPS=600 bash scripts/ab_tunes.sh "" "wt=1" "wt=7" "tail_reduce=0" "head_generic=1" "stack_k16=1" "stack_dbg=128" > gpurun_out/r4_ab1.txt 2>&1 || { cat gpurun_out/r4_ab1.txt; exit 1; }
cat gpurun_out/r4_ab1.txt
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "dense_opt=0" "tail_reduce=0" "wt=7" > gpurun_out/r4_ab_legacy.txt 2>&1 || { cat gpurun_out/r4_ab_legacy.txt; exit 1; }
cat gpurun_out/r4_ab_legacy.txt
INTML_DP_FORCE=1 ROUNDS=2 STEPS=600 bash scripts/ab_tunes.sh "" "dp_early=0" > gpurun_out/r4_ab_dp1.txt 2>&1 || { cat gpurun_out/r4_ab_dp1.txt; exit 1; }
cat gpurun_out/r4_ab_dp1.txt
bash scripts/gpu_r4_prof.sh
