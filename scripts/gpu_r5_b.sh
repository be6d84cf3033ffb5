#!/bin/bash
# Round-5 pass B: the DP workflow tests on the native reducer (no gloo forcing), the fused-dense
# optimizer fallback test, then the driver's exact bench command with the clock settle against
# a 600-step run (and the settle off, for the record).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_integration.py tests/test_convergence.py \
  "tests/test_hip_model.py::test_fused_dense_optimizer_falls_back" > gpurun_out/r5b_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r5b_tests.log | tail -n 30
if [ $rc -ne 0 ]; then tail -n 60 gpurun_out/r5b_tests.log; exit $rc; fi
for i in 1 2; do
  $T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-hpo > gpurun_out/r5b_driver_$i.log 2>&1 || { tail -n 30 gpurun_out/r5b_driver_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5b_driver_$i.log').read().strip().splitlines()[-1]);print('driver-cmd settled', d['value'], d['ms_per_step'], d['settle_steps'], d['settle_ms'])"
  $T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-hpo --settle-ms 0 > gpurun_out/r5b_driver0_$i.log 2>&1 || { tail -n 30 gpurun_out/r5b_driver0_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5b_driver0_$i.log').read().strip().splitlines()[-1]);print('driver-cmd no-settle', d['value'], d['ms_per_step'])"
  $T 200 python bench.py --gpus 1 --steps 600 --warmup 80 --no-hpo > gpurun_out/r5b_long_$i.log 2>&1 || { tail -n 30 gpurun_out/r5b_long_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5b_long_$i.log').read().strip().splitlines()[-1]);print('long 600', d['value'], d['ms_per_step'])"
done
