#!/bin/bash
# Per-launch timings of the conv backward under halo-wgrad split / block knobs (stack_ablate.py).
cd $GRAFT_REPO_ROOT
run() { echo "== $*"; env "$@" timeout -k 10 100 python scripts/stack_ablate.py ${B:-128} 2>&1 | grep -E "wgrad|reduce|sum"; }
run INTML_WGRAD_SPLITS=1024 || exit 1
run INTML_WGRAD_SPLITS=512 || exit 1
run INTML_WGRAD_SPLITS=256 || exit 1
run INTML_WGRAD_SPLITS=2048 || exit 1
run INTML_WGRAD_BLOCK_PX=512 || exit 1
run INTML_WGRAD_BLOCK_PX=128 || exit 1
