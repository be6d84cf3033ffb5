#!/bin/bash
# HPO throughput on the GPU box (via gpurun): the nested HPO x DP GPU test, then
# bench.py --hpo {cray,rpv,mnist}; one JSON line each -> gpurun_out/hpo_bench.jsonl.
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_integration.py -x -v -m gpu -k nested --timeout 280 \
    --timeout-method thread > gpurun_out/nested_test.log 2>&1 || { tail -n 40 gpurun_out/nested_test.log; exit 1; }
tail -n 2 gpurun_out/nested_test.log
H=gpurun_out/hpo_bench.jsonl
: > $H
timeout -k 10 400 python bench.py --hpo cray -- --evals-per-slot 4 2> gpurun_out/hpo_cray.err | grep '^{' >> $H
tail -n 1 $H | cut -c1-300
timeout -k 10 300 python bench.py --hpo rpv 2> gpurun_out/hpo_rpv.err | grep '^{' >> $H
tail -n 1 $H | cut -c1-300
timeout -k 10 300 python bench.py --hpo mnist 2> gpurun_out/hpo_mnist.err | grep '^{' >> $H
tail -n 1 $H | cut -c1-300
