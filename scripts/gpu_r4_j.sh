#!/bin/bash
# Round-4 pass J: evidence on the final kernels -- the four-plane data-plane probe at N=1
# (DP-forced loopback), DP-forced bench, MNIST and legacy kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
INTML_DP_FORCE=1 INTML_PLANE_PROBE=1 $T 400 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/r4j_probe_n1.log 2>&1 || { tail -n 20 gpurun_out/r4j_probe_n1.log; exit 1; }
tail -n 1 gpurun_out/r4j_probe_n1.log | cut -c1-1500
$T 400 python bench.py > gpurun_out/r4j_bench_default.log 2>&1 || { tail -n 20 gpurun_out/r4j_bench_default.log; exit 1; }
tail -n 1 gpurun_out/r4j_bench_default.log | cut -c1-1800
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/r4j_rpv_stats.txt || exit 1
head -14 gpurun_out/r4j_rpv_stats.txt
$T 200 python scripts/stack_timeline.py > gpurun_out/r4j_stack_timeline.txt 2>&1 || { tail -n 20 gpurun_out/r4j_stack_timeline.txt; exit 1; }
$T 200 python scripts/bwd_timeline.py > gpurun_out/r4j_bwd_timeline.txt 2>&1 || { tail -n 20 gpurun_out/r4j_bwd_timeline.txt; exit 1; }
MODEL=mnist bash scripts/prof_model.sh > gpurun_out/r4j_mnist_stats.txt || exit 1
head -16 gpurun_out/r4j_mnist_stats.txt
MODEL=rpv_legacy STEPS=12 WARMUP=3 bash scripts/prof_model.sh > gpurun_out/r4j_legacy_stats.txt || exit 1
head -20 gpurun_out/r4j_legacy_stats.txt
