#!/bin/bash
# Round-4 pass R: dense dX tiles on MNIST / legacy, split-K forward waves on RPV, then the GPU
# suite and the default bench line at the final defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
ROUNDS=2 BENCH_ARGS="--model mnist" bash scripts/ab_tunes.sh "" "dx_min_wgs=512" > gpurun_out/r4r_ab_mnist.txt 2>&1 || { cat gpurun_out/r4r_ab_mnist.txt; exit 1; }
cat gpurun_out/r4r_ab_mnist.txt
ROUNDS=2 STEPS=60 BENCH_ARGS="--model rpv_legacy" bash scripts/ab_tunes.sh "" "dx_min_wgs=512" > gpurun_out/r4r_ab_legacy.txt 2>&1 || { cat gpurun_out/r4r_ab_legacy.txt; exit 1; }
cat gpurun_out/r4r_ab_legacy.txt
ROUNDS=2 STEPS=600 bash scripts/ab_tunes.sh "" "dense_waves=1024" "dense_waves=4096" > gpurun_out/r4r_ab_rpv.txt 2>&1 || { cat gpurun_out/r4r_ab_rpv.txt; exit 1; }
cat gpurun_out/r4r_ab_rpv.txt
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4r_gpu_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/r4r_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
$T 450 python bench.py > gpurun_out/r4r_bench_default.log 2>&1 || { tail -n 20 gpurun_out/r4r_bench_default.log; exit 1; }
tail -n 1 gpurun_out/r4r_bench_default.log | cut -c1-1200
