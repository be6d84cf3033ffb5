#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_hpo.log 2>&1
rc=$?
tail -n 1 gpurun_out/bench_hpo.log > gpurun_out/bench_hpo.json
python -c "import json; d=json.load(open('gpurun_out/bench_hpo.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('hpo')))" || tail -n 30 gpurun_out/bench_hpo.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --batch 1024 --steps 100 --warmup 20 --no-hpo > gpurun_out/bench_b1024.log 2>&1 || { tail -n 20 gpurun_out/bench_b1024.log; exit 1; }
tail -n 1 gpurun_out/bench_b1024.log | cut -c1-200
