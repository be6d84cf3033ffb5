#!/bin/bash
# Full 1-GPU measurement pass (via gpurun): benches, HPO, kernel profiles.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; tail -n 1 gpurun_out/$name.log | tee -a gpurun_out/all.jsonl; }
run bench_rpv 300 python bench.py --steps 200 --warmup 20
run bench_mnist 300 python bench.py --model mnist --steps 100 --warmup 20
run bench_legacy 300 python bench.py --model rpv_legacy --steps 50 --warmup 10
run bench_b1024 300 python bench.py --batch 1024 --steps 100 --warmup 20
run hpo_rpv 400 python benchmarks/hpo_throughput.py --model rpv --trials 32
run hpo_mnist 400 python benchmarks/hpo_throughput.py --model mnist --trials 64
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/prof_rpv_summary.txt
MODEL=rpv_legacy STEPS=10 bash scripts/prof_model.sh > gpurun_out/prof_rpv_legacy_summary.txt
