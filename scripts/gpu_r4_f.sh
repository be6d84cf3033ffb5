#!/bin/bash
# Round-4 pass F: fused dense + head (fence-free hand-off), pipelined standalone wgrad, legacy
# fused dense optimizer: numerics, A/Bs, DP xGMI step at P=2/4/8, legacy stats, profiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py tests/test_dense_bwd.py -m gpu -k "dense_head or wgrad_pipelined or dense_fused or bf16_reference" > gpurun_out/r4f_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4f_numerics.log | head -30
STEPS=600 bash scripts/ab_tunes.sh "" "dense_head=0" "wgrad_dbg=32" > gpurun_out/r4f_ab_rpv.txt 2>&1 || { cat gpurun_out/r4f_ab_rpv.txt; exit 1; }
cat gpurun_out/r4f_ab_rpv.txt
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "dense_opt=0" "wgrad_dbg=32" > gpurun_out/r4f_ab_legacy.txt 2>&1 || { cat gpurun_out/r4f_ab_legacy.txt; exit 1; }
cat gpurun_out/r4f_ab_legacy.txt
$T 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_comm.py -m gpu -k "dp_step_xgmi" > gpurun_out/r4f_comm.log 2>&1
echo "comm rc=$?"; grep -E "PASSED|FAILED|ERROR|AssertionError" gpurun_out/r4f_comm.log | head -20
MODEL=rpv_legacy STEPS=12 WARMUP=3 bash scripts/prof_model.sh > gpurun_out/r4f_legacy_stats.txt || exit 1
head -24 gpurun_out/r4f_legacy_stats.txt
bash scripts/gpu_r4_prof.sh
