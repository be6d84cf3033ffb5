#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
$T 900 $PYT tests -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python scripts/ab_launches.py "lds_layout=1" > gpurun_out/ab_vgpr.txt 2>&1 || { tail -n 20 gpurun_out/ab_vgpr.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_vgpr.txt
for m in rpv mnist; do
$T 300 python bench.py --model $m --steps 200 --warmup 20 --no-hpo > gpurun_out/bench_$m.log 2>&1 || { tail -n 30 gpurun_out/bench_$m.log; exit 1; }
tail -n 1 gpurun_out/bench_$m.log | cut -c1-200
done
$T 300 python bench.py --model rpv_legacy --steps 40 --warmup 10 --no-hpo > gpurun_out/bench_legacy.log 2>&1 || { tail -n 30 gpurun_out/bench_legacy.log; exit 1; }
tail -n 1 gpurun_out/bench_legacy.log | cut -c1-200
MODEL=rpv_legacy STEPS=10 WARMUP=4 bash scripts/prof_model.sh > gpurun_out/prof_legacy_summary.txt || exit 1
head -16 gpurun_out/prof_legacy_summary.txt
