#!/bin/bash
# One build->measure iteration on the GPU box (via gpurun): kernel numerics tests,
# per-launch timing (+ ablations), and the 1-GPU RPV bench.  Stops at the first failure.
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_model.py -x -q -m gpu \
    ${TESTK:+-k "$TESTK"} --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 \
    || { tail -n 40 gpurun_out/iter_tests.log; exit 1; }
tail -n 1 gpurun_out/iter_tests.log
timeout -k 10 120 python scripts/stack_ablate.py > gpurun_out/iter_ablate.txt 2>&1 || { tail -n 20 gpurun_out/iter_ablate.txt; exit 1; }
cat gpurun_out/iter_ablate.txt | grep -v amdgpu.ids
timeout -k 10 120 python bench.py --steps 400 --warmup 40 > gpurun_out/iter_bench.log 2>&1 || { tail -n 20 gpurun_out/iter_bench.log; exit 1; }
tail -n 1 gpurun_out/iter_bench.log | cut -c1-250
