#!/bin/bash
# round 6: MNIST dense tail diagnosis -- head phase stamps (MNIST and RPV) and the MNIST PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MODEL=mnist timeout -k 10 200 python scripts/head_timeline.py > gpurun_out/r6aa_head_mnist.txt 2>&1 || { tail -n 20 gpurun_out/r6aa_head_mnist.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6aa_head_mnist.txt
MODEL=rpv timeout -k 10 200 python scripts/head_timeline.py > gpurun_out/r6aa_head_rpv.txt 2>&1 || { tail -n 20 gpurun_out/r6aa_head_rpv.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6aa_head_rpv.txt
MODEL=mnist TAG=r6aa_mnist bash scripts/gpu_pmc.sh || exit 1
