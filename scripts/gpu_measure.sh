#!/bin/bash
# Measurement sweep for the README / BASELINE tables (one gpurun call):
#   TAG=v7 bash scripts/gpu_measure.sh
# -> gpurun_out/$TAG_benches.jsonl, gpurun_out/$TAG_hpo.jsonl, rocprofv3 kernel stats.
# Each GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-v7}
cd $R
mkdir -p gpurun_out
B=gpurun_out/${TAG}_benches.jsonl
: > $B
run() { timeout -k 10 180 "$@" 2> gpurun_out/${TAG}_last.err | grep '^{' >> $B; tail -n 1 $B | cut -c1-150; }
run python bench.py --steps 400 --warmup 40
INTML_DP_FORCE=1 run python bench.py --steps 400 --warmup 40
run python bench.py --model mnist --steps 400 --warmup 40
run python bench.py --model rpv_legacy --steps 100 --warmup 20
run python bench.py --batch 1024 --steps 100 --warmup 20
H=gpurun_out/${TAG}_hpo.jsonl
: > $H
timeout -k 10 300 python benchmarks/hpo_throughput.py --trials 32 2> gpurun_out/${TAG}_hpo_rpv.err | grep '^{' >> $H
tail -n 1 $H | cut -c1-150
timeout -k 10 300 python benchmarks/hpo_throughput.py --model mnist --trials 64 2> gpurun_out/${TAG}_hpo_mnist.err \
    | grep '^{' >> $H
tail -n 1 $H | cut -c1-150
for m in rpv rpv_legacy; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof_$m -o run -- \
      python $R/bench.py --model $m --steps 24 --warmup 8 > $R/gpurun_out/${TAG}_prof_$m.log 2>&1
  cd $R
  python scripts/prof_summary.py gpurun_out/${TAG}_prof_$m/run_kernel_stats.csv 32 > gpurun_out/${TAG}_${m}_kernel_stats.txt
  head -n 14 gpurun_out/${TAG}_${m}_kernel_stats.txt
done
