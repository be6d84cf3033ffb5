#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_synth.py -x > gpurun_out/synth.log 2>&1 || { tail -n 30 gpurun_out/synth.log; exit 1; }
tail -n 1 gpurun_out/synth.log
timeout -k 10 600 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_hpo.log 2>&1
rc=$?
tail -n 1 gpurun_out/bench_hpo.log > gpurun_out/bench_hpo.json
python -c "import json; d=json.load(open('gpurun_out/bench_hpo.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('hpo')))" || tail -n 30 gpurun_out/bench_hpo.log
exit $rc
