#!/bin/bash
# Round-4 pass K: the dual launch's 3-m-tile instance (bit identity + A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py -m gpu -k "three_mtile" > gpurun_out/r4k_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4k_numerics.log | head
STEPS=600 bash scripts/ab_tunes.sh "" "wgrad_dbg=64" > gpurun_out/r4k_ab_rpv.txt 2>&1 || { cat gpurun_out/r4k_ab_rpv.txt; exit 1; }
cat gpurun_out/r4k_ab_rpv.txt
$T 400 python bench.py > gpurun_out/r4k_bench_default.log 2>&1 || { tail -n 20 gpurun_out/r4k_bench_default.log; exit 1; }
tail -n 1 gpurun_out/r4k_bench_default.log | cut -c1-2500
