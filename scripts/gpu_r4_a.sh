#!/bin/bash
# Round-4 pass A: comm / DP tests (RCCL loopback, xGMI ranks on one GPU, full-step xGMI DP at
# P=2/4/8), the new head / bf16-oracle numerics tests, then the profiling pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -v --timeout 450 --timeout-method thread tests/test_comm.py -m gpu > gpurun_out/r4_comm.log 2>&1
echo "comm rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4_comm.log | head -20
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py -m gpu -k "head_fast or bf16_reference or grads_match_reference" -s > gpurun_out/r4_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR|worst grad" gpurun_out/r4_numerics.log | head -30
bash scripts/gpu_r4_prof.sh
