#!/bin/bash
# xGMI fused all-reduce checks on one GPU: comm tests (2 processes on one GPU via IPC, size-1 DP),
# then the DP-forced bench with the xGMI path.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_comm.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/xgmi_tests.log 2>&1 || { tail -n 60 gpurun_out/xgmi_tests.log; exit 1; }
tail -n 3 gpurun_out/xgmi_tests.log
INTML_XGMI=1 INTML_DP_FORCE=1 timeout -k 10 300 python bench.py > gpurun_out/xgmi_bench.log 2>&1 || { tail -n 30 gpurun_out/xgmi_bench.log; exit 1; }
tail -n 1 gpurun_out/xgmi_bench.log
INTML_DP_FORCE=1 timeout -k 10 300 python bench.py --no-dp-delta > gpurun_out/dpforce_bench.log 2>&1 || { tail -n 30 gpurun_out/dpforce_bench.log; exit 1; }
tail -n 1 gpurun_out/dpforce_bench.log | cut -c1-250
