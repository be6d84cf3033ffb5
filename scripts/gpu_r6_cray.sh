#!/bin/bash
# Round-6 CrayHPO_rpv nested HPO x DP measurement: a genetic search shaped as
# CrayHPO_rpv.ipynb:84-89 (pop 8 x 4 demes; 2 generations instead of 4 so the run fits one GPU
# call), every evaluation a 2-rank data-parallel train_rpv process (4 epochs, 64k / 32k, batch
# 64 per rank) on the native reducer -- the ranks share this box's one GPU, so they run the
# RCCL-free xGMI plane -- with every evaluation's process start-up inside the wall time.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1080 python bench.py --hpo cray -- --generations ${GENS:-2} --demes 4 --pop-size 8 \
  > gpurun_out/r6_cray_hpo.json 2> gpurun_out/r6_cray_hpo.err || { tail -n 30 gpurun_out/r6_cray_hpo.err; exit 1; }
cat gpurun_out/r6_cray_hpo.json
