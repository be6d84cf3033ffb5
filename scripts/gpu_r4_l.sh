#!/bin/bash
# Round-4 pass L: the GPU suite and the default bench line after the farm fix (the inline
# HPO's trials spread over the farm's engines) and the 3-m-tile revert.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4l_gpu_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4l_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
$T 450 python bench.py > gpurun_out/r4l_bench_default.log 2>&1 || { tail -n 20 gpurun_out/r4l_bench_default.log; exit 1; }
tail -n 1 gpurun_out/r4l_bench_default.log | cut -c1-3000
