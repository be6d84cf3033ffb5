#!/bin/bash
# Round-4 pass E: pipelined standalone-wgrad k loop (bit identity + A/B), legacy defaults
# (fused dense optimizer), legacy kernel stats on the current kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py tests/test_dense_bwd.py -m gpu -k "wgrad_pipelined or dense_fused" > gpurun_out/r4e_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4e_numerics.log | head -20
STEPS=600 bash scripts/ab_tunes.sh "" "wgrad_dbg=32" > gpurun_out/r4e_ab_rpv.txt 2>&1 || { cat gpurun_out/r4e_ab_rpv.txt; exit 1; }
cat gpurun_out/r4e_ab_rpv.txt
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "dense_opt=0" "wgrad_dbg=32" > gpurun_out/r4e_ab_legacy.txt 2>&1 || { cat gpurun_out/r4e_ab_legacy.txt; exit 1; }
cat gpurun_out/r4e_ab_legacy.txt
MODEL=rpv_legacy STEPS=12 WARMUP=3 bash scripts/prof_model.sh > gpurun_out/r4e_legacy_stats.txt || exit 1
head -24 gpurun_out/r4e_legacy_stats.txt
