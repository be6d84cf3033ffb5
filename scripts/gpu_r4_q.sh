#!/bin/bash
# Round-4 pass Q: the dense dX at 2 n-tiles per wave (dx_min_wgs 256) -- numerics, A/B against
# 512 / 128 -- and steps per graph 32 against 8 at the new default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_model.py tests/test_dense_bwd.py -m gpu \
  -k "dense_dx_tiles or grads_match or dense_and_head or dense_head or dense_bwd" > gpurun_out/r4q_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4q_tests.log | tail -n 40; tail -n 2 gpurun_out/r4q_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=600 bash scripts/ab_tunes.sh "" "dx_min_wgs=512" "dx_min_wgs=128" > gpurun_out/r4q_ab_rpv.txt 2>&1 || { cat gpurun_out/r4q_ab_rpv.txt; exit 1; }
cat gpurun_out/r4q_ab_rpv.txt
for i in 1 2; do for g in 8 32; do
  r=$($T 120 python bench.py --steps 640 --warmup 64 --no-hpo --steps-per-graph $g 2>/dev/null | tail -n 1) || exit 1
  echo "r$i [spg=$g] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/r4q_spg.txt
