#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
$T 600 $PYT tests/test_hip_kernels.py -x -k "wide or legacy" > gpurun_out/big_tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/big_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python bench.py --model rpv_legacy --steps 40 --warmup 10 --no-hpo > gpurun_out/bench_legacy.log 2>&1 || { tail -n 30 gpurun_out/bench_legacy.log; exit 1; }
tail -n 1 gpurun_out/bench_legacy.log | cut -c1-200
MODEL=rpv_legacy STEPS=10 WARMUP=4 bash scripts/prof_model.sh > gpurun_out/prof_legacy_summary.txt || exit 1
head -16 gpurun_out/prof_legacy_summary.txt
