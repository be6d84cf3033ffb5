#!/bin/bash
# rocprofv3 kernel stats of the bench step for one model: MODEL=rpv_legacy bash scripts/prof_model.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
MODEL=${MODEL:-rpv}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$MODEL -o run -- python $R/bench.py --model $MODEL --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS:---no-hpo} > $R/gpurun_out/prof_$MODEL.log 2>&1 || { echo "prof failed"; tail -n 30 $R/gpurun_out/prof_$MODEL.log; exit 1; }
cd $R && tail -n 1 gpurun_out/prof_$MODEL.log && python scripts/prof_summary.py gpurun_out/prof_$MODEL/run_kernel_stats.csv
