#!/bin/bash
# Full GPU test suite + benches (via gpurun).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -n 60 gpurun_out/full_tests.log; exit 1; }
tail -n 2 gpurun_out/full_tests.log
for m in rpv mnist rpv_legacy; do
  timeout -k 10 300 python bench.py --model $m --steps 100 --warmup 20 > gpurun_out/full_$m.log 2>&1 || { tail -n 20 gpurun_out/full_$m.log; exit 1; }
  tail -n 1 gpurun_out/full_$m.log | cut -c1-200
done
if [ -n "$PROF" ]; then MODEL=$PROF STEPS=10 bash scripts/prof_model.sh > gpurun_out/prof_summary.txt 2>&1; head -n 25 gpurun_out/prof_summary.txt; fi
