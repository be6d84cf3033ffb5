#!/bin/bash
# Round-4 pass A: comm / DP tests (RCCL loopback, xGMI ranks on one GPU, full-step xGMI DP at
# P=2/4/8), the new numerics tests (head fast paths, tail reduction, k16 first layer, bf16
# oracle, fused dense optimizer packs), A/Bs of the new step variants (RPV, legacy), then the
# profiling pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -v --timeout 450 --timeout-method thread tests/test_comm.py -m gpu > gpurun_out/r4_comm.log 2>&1
echo "comm rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4_comm.log | head -20
$T 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py tests/test_dense_bwd.py -m gpu -k "head_fast or tail_reduction or stack_k16 or fast_prologue or bf16_reference or grads_match_reference or dense_fused or write_through" -s > gpurun_out/r4_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR|worst grad" gpurun_out/r4_numerics.log | head -40
