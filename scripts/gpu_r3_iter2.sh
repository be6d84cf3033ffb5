#!/bin/bash
# Round-3 (session 2) iteration pass: model numerics tests, the bench, then an optional
# INTML_TUNE sweep ($TUNES) -- every GPU step under its own time limit, stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -q -x --timeout 180 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py ${EXTRA_TESTS} > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 25 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-260
if [ -n "$TUNES" ]; then bash scripts/gpu_tune_sweep.sh || exit 1; fi
