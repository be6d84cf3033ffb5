#!/bin/bash
# Full GPU pass: the whole -m gpu suite, the three benches, kernel stats of the flagship.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
$T 1000 $PYT tests -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-220
$T 300 python bench.py --model mnist --steps 200 --warmup 20 --no-hpo > gpurun_out/bench_mnist.log 2>&1 || { tail -n 30 gpurun_out/bench_mnist.log; exit 1; }
tail -n 1 gpurun_out/bench_mnist.log | cut -c1-220
$T 300 python bench.py --model rpv_legacy --steps 40 --warmup 10 --no-hpo > gpurun_out/bench_legacy.log 2>&1 || { tail -n 30 gpurun_out/bench_legacy.log; exit 1; }
tail -n 1 gpurun_out/bench_legacy.log | cut -c1-220
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/prof_rpv_summary.txt || exit 1
head -14 gpurun_out/prof_rpv_summary.txt
MODEL=rpv_legacy STEPS=10 WARMUP=4 bash scripts/prof_model.sh > gpurun_out/prof_legacy_summary.txt || exit 1
head -14 gpurun_out/prof_legacy_summary.txt
