#!/bin/bash
# Data-plane probe at N=1 (loopback): INTML_PLANE_PROBE forces the xGMI-vs-RCCL probe.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
INTML_DP_FORCE=1 INTML_PLANE_PROBE=1 timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/probe_n1.log 2>&1 || { tail -n 30 gpurun_out/probe_n1.log; exit 1; }
tail -n 1 gpurun_out/probe_n1.log | cut -c1-1500
