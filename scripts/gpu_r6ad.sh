#!/bin/bash
# round 6: same-box A/B of two builds of the kernel extension (abtmp/_kernels_{old,new}.so:
# before / after the FLAT -> global load fix), interleaved 600-step rounds, RPV and MNIST
set -o pipefail
cd $GRAFT_REPO_ROOT
SO=cori_intml_examples_amd/_kernels.cpython-310-x86_64-linux-gnu.so
T="timeout -k 10"
for r in 1 2 3; do
  for m in rpv mnist; do
    for v in old new; do
      cp abtmp/_kernels_$v.so $SO
      $T 300 python bench.py --model $m --steps 600 --warmup 80 --no-hpo --no-dp-delta > gpurun_out/r6ad.tmp 2>&1 || { tail -n 20 gpurun_out/r6ad.tmp; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6ad.tmp "r$r $m $v" | tee -a gpurun_out/r6ad_ab.txt
    done
  done
done
cp abtmp/_kernels_new.so $SO
