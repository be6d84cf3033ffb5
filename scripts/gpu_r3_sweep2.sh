#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 180 --timeout-method thread"
$T 300 $PYT tests/test_synth.py -x > gpurun_out/synth.log 2>&1
rc=$?; tail -n 15 gpurun_out/synth.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 400 python scripts/ab_launches.py "wgrad_splits=1024" "wgrad_splits=768" "wgrad_splits=640" "wgrad_splits=704" "wgrad_splits=768,wgrad_block_px0=512" "wgrad_splits=768,wgrad_block_px0=384" "wgrad_splits=768,wgrad_max_rows=6" > gpurun_out/sweep_wgrad2.txt 2>&1 || { tail -n 20 gpurun_out/sweep_wgrad2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/sweep_wgrad2.txt
$T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-200
INTML_TUNE=wgrad_splits=768 $T 300 python bench.py --steps 200 --warmup 20 --no-hpo > gpurun_out/bench768.log 2>&1 || { tail -n 30 gpurun_out/bench768.log; exit 1; }
tail -n 1 gpurun_out/bench768.log | cut -c1-200
