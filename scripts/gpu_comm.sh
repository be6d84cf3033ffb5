#!/bin/bash
# Native RCCL engine on one GPU: test, then the headline bench with and without the
# (size-1) data-parallel path captured into the step graph.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_comm.py -x -v --timeout 240 --timeout-method thread > gpurun_out/comm_tests.log 2>&1 || { tail -n 60 gpurun_out/comm_tests.log; exit 1; }
tail -n 3 gpurun_out/comm_tests.log
timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/comm_bench_plain.log 2>&1 || { tail -n 30 gpurun_out/comm_bench_plain.log; exit 1; }
tail -n 1 gpurun_out/comm_bench_plain.log | cut -c1-160
INTML_DP_FORCE=1 timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/comm_bench_dp1.log 2>&1 || { tail -n 30 gpurun_out/comm_bench_dp1.log; exit 1; }
tail -n 1 gpurun_out/comm_bench_dp1.log | cut -c1-160
INTML_DP_FORCE=1 INTML_TUNE=comm_capture=0 timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/comm_bench_dp1_seg.log 2>&1 || { tail -n 30 gpurun_out/comm_bench_dp1_seg.log; exit 1; }
tail -n 1 gpurun_out/comm_bench_dp1_seg.log | cut -c1-160
