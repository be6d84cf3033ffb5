#!/bin/bash
# GPU round-trip: tests, graph-mode bench, rocprofv3 kernel stats.  Each GPU step has its
# own time limit; stops at the first failure.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/tests.log 2>&1
echo "pytest exit $?" >> gpurun_out/tests.log
tail -n 5 gpurun_out/tests.log
timeout -k 10 300 python bench.py --steps 200 --warmup 30 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -n 20 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py --steps 100 --warmup 20 ${BENCH_ARGS} > $R/gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -n 20 $R/gpurun_out/prof.log; exit 1; }
cd $R && python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv 120
