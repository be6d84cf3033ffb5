#!/bin/bash
# Memory-side PMC passes (HBM bytes, L2 hit/miss) of one model's bench step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
MODEL=${MODEL:-rpv}
TAG=${TAG:-r3_$MODEL}
ST=${STEPS:-6}
cd $R && mkdir -p gpurun_out
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_mem1 -o run -- python3 $R/bench.py --model $MODEL --steps $ST --warmup 2 --no-hpo > $R/gpurun_out/${TAG}_mem1.log 2>&1 || { echo "mem1 failed"; tail -n 5 $R/gpurun_out/${TAG}_mem1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_mem2 -o run -- python3 $R/bench.py --model $MODEL --steps $ST --warmup 2 --no-hpo > $R/gpurun_out/${TAG}_mem2.log 2>&1 || { echo "mem2 failed"; tail -n 5 $R/gpurun_out/${TAG}_mem2.log; exit 1; }
cd $R && python scripts/pmc_summary.py gpurun_out/${TAG}_mem1/run_counter_collection.csv gpurun_out/${TAG}_mem2/run_counter_collection.csv > gpurun_out/${TAG}_mem.txt
grep -A1 "conv_gl\|wgrad_gl\|dense_lds\|optim\|slab\|prologue\|conv_halo\|dense_wgrad\|wgrad_halo" gpurun_out/${TAG}_mem.txt | head -40
