#!/bin/bash
# Round-4 pass G: legacy fused dense update without the in-place gradient store, DP xGMI step
# at P=2/4/8, RPV A/Bs at the defaults, profiling pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_dense_bwd.py tests/test_hip_model.py -m gpu -k "dense_fused or dense_head or late_ktab or early_dma or dgrad_onebatch" > gpurun_out/r4g_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4g_numerics.log | head -20
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "opt_nograd=0" > gpurun_out/r4g_ab_legacy.txt 2>&1 || { cat gpurun_out/r4g_ab_legacy.txt; exit 1; }
cat gpurun_out/r4g_ab_legacy.txt
STEPS=600 bash scripts/ab_tunes.sh "" "wgrad_dbg=32" "stack_dbg=256" "dgrad_dbg=64" "early_reduce=0" > gpurun_out/r4g_ab_rpv.txt 2>&1 || { cat gpurun_out/r4g_ab_rpv.txt; exit 1; }
cat gpurun_out/r4g_ab_rpv.txt
$T 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_comm.py -m gpu -k "dp_step_xgmi" > gpurun_out/r4g_comm.log 2>&1
echo "comm rc=$?"; grep -E "PASSED|FAILED|ERROR|AssertionError" gpurun_out/r4g_comm.log | head -20
bash scripts/gpu_r4_prof.sh
