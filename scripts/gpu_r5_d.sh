#!/bin/bash
# Round-5 pass D: the layer-signature-specialised conv stack and the production-only dual
# (wgrad || dgrad) kernels -- bit-identity tests (the A/B forms now run as the generic stack /
# standalone launches) and interleaved bench A/Bs; then the xGMI data plane at N=1 (DP forced):
# its fixed cost per fence form, RCCL, non-DP, and a kernel trace of the xGMI step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
# (no -x: a bit-identity failure is reported, the measurements below still run; a crash or a
# timeout stops the script)
$T 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_hip_model.py tests/test_comm.py \
  > gpurun_out/r5d_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|ERROR" gpurun_out/r5d_tests.log | tail -n 12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -n 60 gpurun_out/r5d_tests.log; exit $rc; fi
grep -A12 "^E  " gpurun_out/r5d_tests.log | head -40
ROUNDS=3 STEPS=600 bash scripts/ab_tunes.sh "" "stack_spec=0" > gpurun_out/r5d_ab_rpv.txt 2>&1 || { cat gpurun_out/r5d_ab_rpv.txt; exit 1; }
cat gpurun_out/r5d_ab_rpv.txt
ROUNDS=2 STEPS=600 BENCH_ARGS="--model mnist" bash scripts/ab_tunes.sh "" "stack_spec=0" > gpurun_out/r5d_ab_mnist.txt 2>&1 || { cat gpurun_out/r5d_ab_mnist.txt; exit 1; }
cat gpurun_out/r5d_ab_mnist.txt
run() {   # tag, env...
  local tag=$1; shift
  env "$@" $T 200 python bench.py --steps 400 --warmup 40 --no-hpo --no-dp-delta > gpurun_out/r5d_$tag.log 2>&1 || { tail -n 30 gpurun_out/r5d_$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5d_$tag.log').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'], (d.get('selfcheck') or {}).get('data_plane'))"
}
run nodp || exit 1
for f in 2 1 0; do run dp1_xgmi_f$f INTML_DP_FORCE=1 INTML_XGMI=xgmi INTML_TUNE=xgmi_fence=$f || exit 1; done
run dp1_rccl INTML_DP_FORCE=1 INTML_XGMI=rccl || exit 1
run nodp_b || exit 1
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/r5d_rpv_stats.txt || exit 1
head -14 gpurun_out/r5d_rpv_stats.txt
INTML_DP_FORCE=1 INTML_XGMI=xgmi MODEL=rpv BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > gpurun_out/r5d_xgmi_stats.txt || exit 1
head -14 gpurun_out/r5d_xgmi_stats.txt
