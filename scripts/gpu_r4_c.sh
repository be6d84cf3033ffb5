#!/bin/bash
# Round-4 pass C: DP xGMI step at P=2/4/8 on one GPU (shared-GPU grid), dgrad one-batch
# prologue (bit identity + A/B), legacy fused dense optimizer A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py -m gpu -k "dgrad_onebatch or write_through" > gpurun_out/r4c_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4c_numerics.log | head -20
STEPS=600 bash scripts/ab_tunes.sh "" "dgrad_dbg=32" > gpurun_out/r4c_ab_rpv.txt 2>&1 || { cat gpurun_out/r4c_ab_rpv.txt; exit 1; }
cat gpurun_out/r4c_ab_rpv.txt
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "dense_opt=auto" > gpurun_out/r4c_ab_legacy.txt 2>&1 || { cat gpurun_out/r4c_ab_legacy.txt; exit 1; }
cat gpurun_out/r4c_ab_legacy.txt
$T 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_comm.py -m gpu -k "dp_step_xgmi" > gpurun_out/r4c_comm.log 2>&1
echo "comm rc=$?"; grep -E "PASSED|FAILED|ERROR|\"error\"" gpurun_out/r4c_comm.log | head -20
