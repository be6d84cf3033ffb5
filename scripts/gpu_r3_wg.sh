#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py -x > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 2 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 200 python scripts/bwd_timeline.py > gpurun_out/bwd_timeline.txt 2>&1 || { tail -n 20 gpurun_out/bwd_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bwd_timeline.txt | grep "span\|phases\|wgrad start\|dgrad start" | head -20
$T 300 python scripts/ab_launches.py "lds_layout=1" > gpurun_out/ab_wg.txt 2>&1 || { tail -n 20 gpurun_out/ab_wg.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_wg.txt
$T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-200
