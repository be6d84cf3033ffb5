#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py -x -k "stack" > gpurun_out/stack_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/stack_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 200 python scripts/stack_timeline.py > gpurun_out/stack_timeline.txt 2>&1 || { tail -n 20 gpurun_out/stack_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stack_timeline.txt | tail -n 17
$T 300 python scripts/ab_launches.py "conv_stack=1" > gpurun_out/ab_stack.txt 2>&1 || { tail -n 20 gpurun_out/ab_stack.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_stack.txt
$T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-200
