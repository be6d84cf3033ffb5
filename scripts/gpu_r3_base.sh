#!/bin/bash
# Round-3 pass: GPU tests, 1-GPU bench, kernel stats of the bench step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -n 30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/prof_rpv_summary.txt || exit 1
head -20 gpurun_out/prof_rpv_summary.txt
