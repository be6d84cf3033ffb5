#!/bin/bash
# Round-4 pass T: dense wgrad at 4 n-tiles as the default -- legacy A/B, the GPU suite, the
# default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "dw_ntt=8" > gpurun_out/r4t_ab_legacy.txt 2>&1 || { cat gpurun_out/r4t_ab_legacy.txt; exit 1; }
cat gpurun_out/r4t_ab_legacy.txt
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4t_gpu_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/r4t_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
$T 450 python bench.py > gpurun_out/r4t_bench_default.log 2>&1 || { tail -n 20 gpurun_out/r4t_bench_default.log; exit 1; }
tail -n 1 gpurun_out/r4t_bench_default.log | cut -c1-600
