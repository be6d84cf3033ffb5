#!/bin/bash
# Round-4 pass B: comm/DP tests (xGMI DP step at P=2/4/8 with timeout diagnostics), the
# numerics tests of this round's step variants, A/Bs of the new defaults, profiling pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_comm.py -m gpu > gpurun_out/r4b_comm.log 2>&1
echo "comm rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4b_comm.log | head -20
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py tests/test_dense_bwd.py -m gpu -k "head_fast or stack_k16 or fast_prologue or bf16_reference or dense_fused or write_through" > gpurun_out/r4b_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4b_numerics.log | head -20
STEPS=600 bash scripts/ab_tunes.sh "" "wt=0" "stack_k16=0" > gpurun_out/r4b_ab_rpv.txt 2>&1 || { cat gpurun_out/r4b_ab_rpv.txt; exit 1; }
cat gpurun_out/r4b_ab_rpv.txt
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "wt=0" > gpurun_out/r4b_ab_legacy.txt 2>&1 || { cat gpurun_out/r4b_ab_legacy.txt; exit 1; }
cat gpurun_out/r4b_ab_legacy.txt
INTML_DP_FORCE=1 ROUNDS=2 STEPS=600 bash scripts/ab_tunes.sh "" "dp_early=0" > gpurun_out/r4b_ab_dp1.txt 2>&1 || { cat gpurun_out/r4b_ab_dp1.txt; exit 1; }
cat gpurun_out/r4b_ab_dp1.txt
bash scripts/gpu_r4_prof.sh
