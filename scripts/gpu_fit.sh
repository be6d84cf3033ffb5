#!/bin/bash
# Recipe-path (fit) vs train_steps bench at B=128 (via gpurun), plain and Horovod-wrapped (DP at N=1).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/fit_ab.jsonl
run() { timeout -k 10 300 env "$@" > gpurun_out/fit_one.log 2>&1 || { tail -n 30 gpurun_out/fit_one.log; exit 1; }; tail -n 1 gpurun_out/fit_one.log >> gpurun_out/fit_ab.jsonl; tail -n 1 gpurun_out/fit_one.log | cut -c1-160; }
run X=1 python bench.py --steps 400 --warmup 40 --no-dp-delta
run X=1 python bench.py --via-fit --fit-epochs 4 --samples 65536
run INTML_DP_FORCE=1 INTML_XGMI=0 python bench.py --steps 400 --warmup 40 --no-dp-delta
run INTML_DP_FORCE=1 INTML_XGMI=0 python bench.py --via-fit --fit-epochs 4 --samples 65536
run INTML_DP_FORCE=1 INTML_XGMI=0 python bench.py --via-fit --fit-epochs 4 --samples 65536 --lr-warmup-epochs 2
