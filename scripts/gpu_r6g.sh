#!/bin/bash
# round 6: the branch-free wgrad fragment reads (wave-uniform m-tile conditions) -- GPU suite,
# RPV / MNIST / legacy 600-step lines, RPV kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TESTS=all TAG=r6g AB_ROUNDS=3 AB_STEPS=600 AB="" PROF="rpv"
bash scripts/gpu_pass.sh || exit 1
for m in mnist rpv_legacy; do
  timeout -k 10 300 python bench.py --model $m --steps 200 --warmup 30 --no-hpo --no-dp-delta > gpurun_out/r6g_$m.log 2>&1 || { tail -n 20 gpurun_out/r6g_$m.log; exit 1; }
  tail -n 1 gpurun_out/r6g_$m.log | cut -c1-300
done
