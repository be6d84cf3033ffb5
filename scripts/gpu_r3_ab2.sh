#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 180 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py -x > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 5 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python scripts/ab_launches.py "lds_layout=0" "lds_layout=1" > gpurun_out/ab_rpv.txt 2>&1 || { tail -n 20 gpurun_out/ab_rpv.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_rpv.txt
$T 300 python scripts/ab_launches.py "lds_layout=0" "lds_layout=1" --model mnist > gpurun_out/ab_mnist.txt 2>&1 || { tail -n 20 gpurun_out/ab_mnist.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_mnist.txt
$T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-200
$T 300 python bench.py --model mnist --steps 200 --warmup 20 --no-hpo > gpurun_out/bench_mnist.log 2>&1 || { tail -n 30 gpurun_out/bench_mnist.log; exit 1; }
tail -n 1 gpurun_out/bench_mnist.log | cut -c1-200
