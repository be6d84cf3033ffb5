#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 180 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py -x > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 3 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
INTML_TUNE=wgrad_perm=0 $T 600 $PYT tests/test_hip_model.py -x -k "grads or stack or steps" > gpurun_out/numerics_perm0.log 2>&1
rc=$?; tail -n 2 gpurun_out/numerics_perm0.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python scripts/ab_launches.py "wgrad_perm=1" "wgrad_perm=0" "wgrad_perm=0,lds_layout=0" > gpurun_out/ab_perm.txt 2>&1 || { tail -n 20 gpurun_out/ab_perm.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_perm.txt
$T 200 python scripts/stack_timeline.py > gpurun_out/stack_timeline.txt 2>&1; grep -v amdgpu.ids gpurun_out/stack_timeline.txt | tail -n 40
$T 200 python scripts/stack_ablate.py > gpurun_out/stack_ablate.txt 2>&1; grep -v amdgpu.ids gpurun_out/stack_ablate.txt | tail -n 15
