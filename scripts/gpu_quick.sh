#!/bin/bash
# Quick GPU check (via gpurun): kernel tests matching $TESTK, then the 1-GPU benches.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py tests/test_hip_model.py -x -q -m gpu ${TESTK:+-k "$TESTK"} > gpurun_out/quick_tests.log 2>&1 || { tail -n 40 gpurun_out/quick_tests.log; exit 1; }
tail -n 2 gpurun_out/quick_tests.log
for m in rpv mnist rpv_legacy; do
  timeout -k 10 300 python bench.py --model $m --steps 100 --warmup 20 > gpurun_out/quick_$m.log 2>&1 || { tail -n 20 gpurun_out/quick_$m.log; exit 1; }
  tail -n 1 gpurun_out/quick_$m.log | cut -c1-200
done
timeout -k 10 300 python bench.py --batch 1024 --steps 50 --warmup 10 > gpurun_out/quick_b1024.log 2>&1 && tail -n 1 gpurun_out/quick_b1024.log | cut -c1-200
if [ -n "$PROF" ]; then MODEL=$PROF STEPS=10 bash scripts/prof_model.sh > gpurun_out/prof_summary.txt 2>&1; head -n 25 gpurun_out/prof_summary.txt; fi
