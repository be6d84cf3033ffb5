#!/bin/bash
# Round-4 pass H: back at the pass-F kernels + the dense dX mask prefetch: numerics, A/B,
# smoke, default bench line (with the HPO records), profiling pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_hip_model.py -m gpu -k "dense_dx_mask or head_fast or bf16_reference" > gpurun_out/r4h_numerics.log 2>&1
echo "numerics rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4h_numerics.log | head -20
STEPS=600 bash scripts/ab_tunes.sh "" "dense_dbg=1" > gpurun_out/r4h_ab_rpv.txt 2>&1 || { cat gpurun_out/r4h_ab_rpv.txt; exit 1; }
cat gpurun_out/r4h_ab_rpv.txt
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h_smoke.log 2>&1 || { tail -n 20 gpurun_out/r4h_smoke.log; exit 1; }
echo "smoke ok"
$T 400 python bench.py > gpurun_out/r4h_bench_default.log 2>&1 || { tail -n 20 gpurun_out/r4h_bench_default.log; exit 1; }
tail -n 1 gpurun_out/r4h_bench_default.log | cut -c1-2000
bash scripts/gpu_r4_prof.sh
