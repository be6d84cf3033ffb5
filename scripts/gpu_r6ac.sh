#!/bin/bash
# round 6: global-address-space loads where the compiler emitted FLAT loads (pointer selects in
# the halo staging, dataset pointers read from the step state): numerics + per-model lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6ac
export TESTS="tests/test_hip_kernels.py tests/test_hip_model.py tests/test_dense_bwd.py"
bash scripts/gpu_pass.sh || exit 1
T="timeout -k 10"
for m in rpv mnist rpv_legacy; do
  st=600; [ $m = rpv_legacy ] && st=150
  for r in 1 2; do
    $T 300 python bench.py --model $m --steps $st --warmup 80 --no-hpo --no-dp-delta > gpurun_out/r6ac_$m.log 2>&1 || { tail -n 20 gpurun_out/r6ac_$m.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6ac_$m.log "$m r$r" | tee -a gpurun_out/r6ac_lines.txt
  done
done
for m in rpv mnist; do
  MODEL=$m STEPS=20 WARMUP=5 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r6ac_${m}_stats.txt || exit 1
  python scripts/prof_sequence.py gpurun_out/prof_$m/run_kernel_trace.csv > gpurun_out/r6ac_${m}_sequence.txt
  cat gpurun_out/r6ac_${m}_sequence.txt
done
