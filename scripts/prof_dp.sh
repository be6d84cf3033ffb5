#!/bin/bash
# rocprofv3 kernel trace of the DP-forced N=1 bench step (RCCL in the graph) + timeline of the last steps.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && INTML_DP_FORCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dp -o run -- python $R/bench.py --steps 16 --warmup 8 --no-dp-delta ${BENCH_ARGS} > $R/gpurun_out/prof_dp.log 2>&1 || { echo "prof failed"; tail -n 30 $R/gpurun_out/prof_dp.log; exit 1; }
cd $R && tail -n 1 gpurun_out/prof_dp.log | cut -c1-300 && python scripts/prof_summary.py gpurun_out/prof_dp/run_kernel_stats.csv 24 > gpurun_out/prof_dp_summary.txt && python scripts/prof_timeline.py gpurun_out/prof_dp/run_kernel_trace.csv 60 > gpurun_out/prof_dp_timeline.txt
