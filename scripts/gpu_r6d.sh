#!/bin/bash
# round 6 profile pass: rocprofv3 kernel stats + per-launch step sequences (prof_sequence.py)
# of the RPV step at B=128 and B=1024 and of the legacy model
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in "rpv:128:r6_rpv" "rpv:1024:r6_rpv_b1024" "rpv_legacy:128:r6_legacy"; do
  IFS=: read m b tag <<< "$spec"
  MODEL=$m STEPS=${STEPS:-20} WARMUP=5 BENCH_ARGS="--no-hpo --no-dp-delta --batch $b" bash scripts/prof_model.sh > gpurun_out/${tag}_kernel_stats.txt || { cat gpurun_out/${tag}_kernel_stats.txt; exit 1; }
  python scripts/prof_sequence.py gpurun_out/prof_$m/run_kernel_trace.csv > gpurun_out/${tag}_sequence.txt || exit 1
  rm -rf gpurun_out/prof_${tag}; mv gpurun_out/prof_$m gpurun_out/prof_${tag}
  head -n 14 gpurun_out/${tag}_kernel_stats.txt; cat gpurun_out/${tag}_sequence.txt
done
