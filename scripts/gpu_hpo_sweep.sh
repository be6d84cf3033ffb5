#!/bin/bash
# HPO throughput sweep on one GPU: engines per GPU x model (run via gpurun).
set -e
mkdir -p gpurun_out
for m in "mnist 64 1" "mnist 64 4" "mnist 64 8" "rpv 16 1" "rpv 16 2" "rpv 24 4"; do
  set -- $m
  timeout -k 10 420 python benchmarks/hpo_throughput.py --model $1 --trials $2 --engines-per-gpu $3 \
      > gpurun_out/hpo_$1_e$3.log 2>&1
  tail -n 1 gpurun_out/hpo_$1_e$3.log
done
