#!/bin/bash
# round 6: the Keras fit() recipe path (apps.rpv.train_model, 4 epochs, the first untimed)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --via-fit --no-hpo --no-dp-delta > gpurun_out/r6ag_fit.log 2>&1 || { tail -n 30 gpurun_out/r6ag_fit.log; exit 1; }
tail -n 1 gpurun_out/r6ag_fit.log | cut -c1-600
