#!/bin/bash
# Per-launch timings of the dense backward under a few executor knobs (stack_ablate.py).
cd $GRAFT_REPO_ROOT
run() { echo "== $*"; env "$@" timeout -k 10 100 python scripts/stack_ablate.py $B 2>&1 | grep -E "dense|reduce|sum"; }
for B in ${BATCHES:-128}; do
  export B
  run INTML_DUAL_DENSE=0 INTML_DENSE_OPT=0 || exit 1
  run INTML_DUAL_DENSE=0 INTML_DENSE_OPT=1 || exit 1
  run INTML_DUAL_DENSE=1 INTML_DENSE_OPT=0 || exit 1
done
