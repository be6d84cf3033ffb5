#!/bin/bash
# Round-4 pass D: numerics of this round's step variants (fused dense + head, dgrad one-batch
# prologue, write-through stores, head paths, bf16 oracle), RPV A/Bs, DP xGMI step at
# P=2/4/8 on one GPU, then the profiling pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py -m gpu -k "dense_head or dgrad_onebatch or write_through or head_fast or bf16_reference" > gpurun_out/r4d_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4d_numerics.log | head -30
STEPS=600 bash scripts/ab_tunes.sh "" "dense_head=0" "dgrad_dbg=32" > gpurun_out/r4d_ab_rpv.txt 2>&1 || { cat gpurun_out/r4d_ab_rpv.txt; exit 1; }
cat gpurun_out/r4d_ab_rpv.txt
$T 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_comm.py -m gpu -k "dp_step_xgmi" > gpurun_out/r4d_comm.log 2>&1
echo "comm rc=$?"; grep -E "PASSED|FAILED|ERROR|\"error\"" gpurun_out/r4d_comm.log | head -20
bash scripts/gpu_r4_prof.sh
