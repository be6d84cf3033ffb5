#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 180 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py -x -k "stack or grads or steps" > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 2 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
$T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-200
done
INTML_TUNE=wgrad_fast=0 $T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench_f0.log 2>&1 || { tail -n 30 gpurun_out/bench_f0.log; exit 1; }
tail -n 1 gpurun_out/bench_f0.log | cut -c1-200
$T 200 python scripts/stack_timeline.py > gpurun_out/stack_timeline.txt 2>&1 || { tail -n 20 gpurun_out/stack_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stack_timeline.txt | tail -n 17
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/prof_rpv_summary.txt || exit 1
head -24 gpurun_out/prof_rpv_summary.txt
