#!/bin/bash
# Generic GPU measurement pass -- the one script every gpurun call goes through (replaces the
# one-off per-round pass scripts; scripts/PASSES.md lists what each past pass ran).  Steps run
# in this order, each only if its variable is set, each under its own time limit; a crash, a
# timeout or a failed test stops the pass (TESTS_CONTINUE=1: a failed test is reported and the
# measurements still run):
#   TESTS="<pytest args>"     e.g. "tests/test_hip_model.py -k 'spec or dual'"  (or "all" = -m gpu)
#   SMOKE=1                   __graft_entry__.smoke()
#   DRIVER=1                  the driver's exact bench command (bench.py --gpus 1 --steps 20 --warmup 5)
#   AB="a|b|c"                interleaved bench A/B of INTML_TUNE variants ("" = defaults), with
#                             AB_MODEL (rpv), AB_STEPS (600), AB_ROUNDS (3), AB_ENV (extra env),
#                             AB_ARGS (extra bench.py flags, e.g. "--batch 1024");
#                             a variant "ENV=v ENV2=w;tune" also sets environment for that arm
#   BENCH="<bench args>"      one bench.py line (BENCH_ENV: extra env)
#   PROF="rpv mnist ..."      rocprofv3 kernel stats of each model's bench step (PROF_ENV)
#   PMC=<model>               the two PMC counter passes of that model (gpu_pmc.sh)
#   TIMELINES=1               in-kernel phase stamps (stack / backward / head timelines)
#   TAG=<name>                prefix of the outputs under gpurun_out/ (default: pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
TAG=${TAG:-pass}
O=gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  if [ "$TESTS" = "all" ]; then TESTS="tests -m gpu"; fi
  eval "$T ${TESTS_LIMIT:-900} python -u -m pytest -v --timeout 200 --timeout-method thread $TESTS" > ${O}_tests.log 2>&1
  rc=$?; grep -E "passed|failed" ${O}_tests.log | tail -n 2; grep -E "FAILED|ERROR" ${O}_tests.log | head -n 20
  if [ $rc -ne 0 ]; then
    grep -B2 -A14 "^E  " ${O}_tests.log | head -n 60
    if [ $rc -ne 1 ] || [ -z "$TESTS_CONTINUE" ]; then exit $rc; fi
  fi
fi
if [ -n "$SMOKE" ]; then
  $T 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 || { tail -n 20 ${O}_smoke.log; exit 1; }
  tail -n 1 ${O}_smoke.log
fi
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('settle_steps'), (d.get('selfcheck') or {}).get('data_plane'))" "$@"; }
if [ -n "$DRIVER" ]; then
  $T 400 python bench.py --gpus 1 --steps 20 --warmup 5 > ${O}_driver.log 2>&1 || { tail -n 30 ${O}_driver.log; exit 1; }
  tail -n 1 ${O}_driver.log | cut -c1-3000
fi
if [ -n "$AB" ]; then
  IFS='|' read -ra VARIANTS <<< "$AB"
  for i in $(seq 1 ${AB_ROUNDS:-3}); do
    for v in "${VARIANTS[@]}"; do
      venv=""; tv="$v"
      if [[ "$v" == *";"* ]]; then venv="${v%%;*}"; tv="${v#*;}"; fi
      env $AB_ENV $venv INTML_TUNE="$tv" $T 200 python bench.py --model ${AB_MODEL:-rpv} --steps ${AB_STEPS:-600} --warmup 80 --no-hpo --no-dp-delta $AB_ARGS \
        > ${O}_ab.tmp 2>&1 || { tail -n 30 ${O}_ab.tmp; exit 1; }
      line ${O}_ab.tmp "r$i [${v:-default}]" | tee -a ${O}_ab.txt
    done
  done
fi
if [ -n "$BENCH" ]; then
  env $BENCH_ENV $T 400 python bench.py $BENCH > ${O}_bench.log 2>&1 || { tail -n 30 ${O}_bench.log; exit 1; }
  line ${O}_bench.log "bench [$BENCH]"
fi
for m in $PROF; do
  env $PROF_ENV MODEL=$m STEPS=${PROF_STEPS:-20} WARMUP=5 bash scripts/prof_model.sh > ${O}_${m}_stats.txt || { cat ${O}_${m}_stats.txt; exit 1; }
  head -n 14 ${O}_${m}_stats.txt
done
if [ -n "$PMC" ]; then
  MODEL=$PMC TAG=${TAG}_$PMC bash scripts/gpu_pmc.sh || exit 1
fi
if [ -n "$TIMELINES" ]; then
  for s in stack bwd head; do
    $T 200 python scripts/${s}_timeline.py > ${O}_${s}_timeline.txt 2>&1 || { tail -n 20 ${O}_${s}_timeline.txt; exit 1; }
  done
  grep -v amdgpu.ids ${O}_stack_timeline.txt | head -n 30
fi
echo "pass $TAG done"
