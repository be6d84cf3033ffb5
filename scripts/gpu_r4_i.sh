#!/bin/bash
# Round-4 pass I: the whole GPU test suite on the final kernels, then evidence: PMC counters of
# the RPV step, the four-plane data-plane probe at N=1 (DP-forced loopback), MNIST and legacy
# kernel stats.  Every step under its own limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4i_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -n 3 gpurun_out/r4i_gpu_tests.log; grep -E "FAILED|ERROR" gpurun_out/r4i_gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
MODEL=rpv TAG=r4_rpv bash scripts/gpu_pmc.sh > gpurun_out/r4i_pmc.out 2>&1 || { tail -n 20 gpurun_out/r4i_pmc.out; exit 1; }
tail -n 40 gpurun_out/r4i_pmc.out
