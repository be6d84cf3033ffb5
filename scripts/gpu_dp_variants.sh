#!/bin/bash
# DP-forced N=1 step variants: comm fork (overlap) vs linear graph vs single bucket.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { name=$1; shift; env "$@" INTML_DP_FORCE=1 timeout -k 10 300 python bench.py --no-dp-delta > gpurun_out/var_$name.log 2>&1 || { tail -n 30 gpurun_out/var_$name.log; exit 1; }; echo "$name $(tail -n 1 gpurun_out/var_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["step_ms_p50"])')"; }
run fork INTML_COMM_FORK=1
run linear INTML_COMM_FORK=0
run linear_1bucket INTML_COMM_FORK=0 INTML_BUCKET_BYTES=1073741824
run fork_1bucket INTML_COMM_FORK=1 INTML_BUCKET_BYTES=1073741824
timeout -k 10 300 python bench.py --no-dp-delta > gpurun_out/var_nodp.log 2>&1 && echo "nodp $(tail -n 1 gpurun_out/var_nodp.log | cut -c1-160)"
export TMPDIR=/tmp
cd /tmp && INTML_COMM_FORK=0 INTML_DP_FORCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_lin -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 16 --warmup 8 --no-dp-delta > $GRAFT_REPO_ROOT/gpurun_out/prof_lin.log 2>&1
cd $GRAFT_REPO_ROOT && python scripts/prof_timeline.py gpurun_out/prof_lin/run_kernel_trace.csv 60 > gpurun_out/prof_lin_timeline.txt
