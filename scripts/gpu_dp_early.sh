#!/bin/bash
# DP-path checks after a data-plane change: the native-comm GPU test, DP-vs-single equivalence,
# and the DP bench at N=1 with / without the early reduce-only groups (interleaved).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_comm.py -m gpu > gpurun_out/comm_tests.log 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || { tail -n 4 gpurun_out/comm_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
[ -n "$SKIP_TESTS" ] || timeout -k 10 240 python scripts/dp_equiv_check.py 1 2>&1 | grep seed || exit 1
: > gpurun_out/dp_early.txt
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/dpe.log 2>&1 || { tail -n 20 gpurun_out/dpe.log; exit 1; }
  echo "r$r non-DP $(tail -n 1 gpurun_out/dpe.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a gpurun_out/dp_early.txt
  for tv in "" "dp_early_reduce=0"; do
    INTML_DP_FORCE=1 INTML_TUNE="$tv" timeout -k 10 180 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/dpe.log 2>&1 || { tail -n 20 gpurun_out/dpe.log; exit 1; }
    echo "r$r DP [$tv] $(tail -n 1 gpurun_out/dpe.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a gpurun_out/dp_early.txt
  done
done
