#!/bin/bash
# N=1 data-plane overheads: plain step vs the forced data-parallel step, and the plane probe
# (xgmi / rccl / rccl_forked / hybrid) in loopback; plus the numerics of the refactored plan.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py tests/test_synth.py -x > gpurun_out/numerics.log 2>&1
rc=$?; tail -n 2 gpurun_out/numerics.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/b_plain.log 2>&1 || { tail -n 30 gpurun_out/b_plain.log; exit 1; }
tail -n 1 gpurun_out/b_plain.log | cut -c1-170
INTML_DP_FORCE=1 $T 300 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/b_dp.log 2>&1 || { tail -n 30 gpurun_out/b_dp.log; exit 1; }
tail -n 1 gpurun_out/b_dp.log | cut -c1-170
INTML_DP_FORCE=1 INTML_PLANE_PROBE=1 $T 400 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/b_probe.log 2>&1 || { tail -n 30 gpurun_out/b_probe.log; exit 1; }
tail -n 1 gpurun_out/b_probe.log > gpurun_out/b_probe.json
python -c "import json; d=json.load(open('gpurun_out/b_probe.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('config',{}).get('plane_probe', d.get('plane_probe'))))"
