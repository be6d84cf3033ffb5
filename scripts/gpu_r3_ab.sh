#!/bin/bash
# Numerics of the kernel paths + per-launch A/B of tune variants + bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 180 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py tests/test_comm.py -x > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 15 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python scripts/ab_launches.py ${AB_VARIANTS:-"lds_layout=0,conv_kpipe=0" "lds_layout=1,conv_kpipe=0" "lds_layout=1,conv_kpipe=1"} > gpurun_out/ab.txt 2>&1 || { tail -n 20 gpurun_out/ab.txt; exit 1; }
cat gpurun_out/ab.txt | grep -v amdgpu.ids
$T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-300
