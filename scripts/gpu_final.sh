#!/bin/bash
# Round-end measurement pass (via gpurun): full GPU test suite, rocprof evidence (gpu_evidence.sh)
# and the benchmark set, each step under its own time limit; stops at the first failure.
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-v12}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
tail -n 1 gpurun_out/${T}_gpu_tests.log
TAG=$T bash scripts/gpu_evidence.sh > gpurun_out/${T}_evidence.log 2>&1
B=gpurun_out/${T}_benches.jsonl; : > $B
timeout -k 10 150 python bench.py --steps 800 --warmup 80 | tail -n 1 >> $B
INTML_DP_FORCE=1 timeout -k 10 150 python bench.py --steps 800 --warmup 80 | tail -n 1 >> $B
timeout -k 10 150 python bench.py --model mnist --steps 800 --warmup 80 | tail -n 1 >> $B
timeout -k 10 200 python bench.py --model rpv_legacy --steps 100 --warmup 20 | tail -n 1 >> $B
timeout -k 10 150 python bench.py --batch 1024 --steps 200 --warmup 20 | tail -n 1 >> $B
cut -c1-150 $B
