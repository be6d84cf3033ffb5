#!/bin/bash
# Round-2 DP / recipe-path check (via gpurun): GPU tests, then bench variants:
# default N=1, DP-forced N=1 (full DP step with RCCL in the graph), fit path with and without LR warmup.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/dp_tests.log 2>&1 || { tail -n 60 gpurun_out/dp_tests.log; exit 1; }
tail -n 2 gpurun_out/dp_tests.log
timeout -k 10 300 python bench.py > gpurun_out/dp_b_default.log 2>&1 || { tail -n 30 gpurun_out/dp_b_default.log; exit 1; }
tail -n 1 gpurun_out/dp_b_default.log
INTML_DP_FORCE=1 timeout -k 10 300 python bench.py > gpurun_out/dp_b_force.log 2>&1 || { tail -n 30 gpurun_out/dp_b_force.log; exit 1; }
tail -n 1 gpurun_out/dp_b_force.log
timeout -k 10 300 python bench.py --via-fit > gpurun_out/dp_b_fit0.log 2>&1 || { tail -n 30 gpurun_out/dp_b_fit0.log; exit 1; }
tail -n 1 gpurun_out/dp_b_fit0.log
timeout -k 10 300 python bench.py --via-fit --lr-warmup-epochs 2 > gpurun_out/dp_b_fit2.log 2>&1 || { tail -n 30 gpurun_out/dp_b_fit2.log; exit 1; }
tail -n 1 gpurun_out/dp_b_fit2.log
INTML_DP_FORCE=1 timeout -k 10 300 python bench.py --via-fit --lr-warmup-epochs 2 > gpurun_out/dp_b_fit2dp.log 2>&1 || { tail -n 30 gpurun_out/dp_b_fit2dp.log; exit 1; }
tail -n 1 gpurun_out/dp_b_fit2dp.log
