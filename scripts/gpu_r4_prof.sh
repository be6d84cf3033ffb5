#!/bin/bash
# Round-4 profiling pass of the RPV bench step: a bench line, rocprofv3 kernel stats, and the
# in-kernel phase timelines (conv stack, head, backward launches) -- each step time-limited,
# stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/r4p_bench.log 2>&1 || { tail -n 30 gpurun_out/r4p_bench.log; exit 1; }
tail -n 1 gpurun_out/r4p_bench.log | cut -c1-240
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/r4p_rpv_stats.txt || exit 1
head -14 gpurun_out/r4p_rpv_stats.txt
$T 200 python scripts/bwd_timeline.py > gpurun_out/r4p_bwd_timeline.txt 2>&1 || { tail -n 20 gpurun_out/r4p_bwd_timeline.txt; exit 1; }
$T 200 python scripts/head_timeline.py > gpurun_out/r4p_head_timeline.txt 2>&1 || { tail -n 20 gpurun_out/r4p_head_timeline.txt; exit 1; }
$T 200 python scripts/stack_timeline.py > gpurun_out/r4p_stack_timeline.txt 2>&1 || { tail -n 20 gpurun_out/r4p_stack_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4p_bwd_timeline.txt | head -30
echo done
