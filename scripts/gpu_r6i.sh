#!/bin/bash
# round 6: full GPU suite + smoke + driver command + exchange / plane A/B + RPV kernel stats at the
# current kernels (wgrad loop + dual extras reduced to modes 1 / 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TESTS=all SMOKE=1 DRIVER=1 TAG=r6i AB_ROUNDS=3 AB_STEPS=600 PROF="rpv"
export AB="|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xchg_p1=1|INTML_DP_FORCE=1 INTML_XGMI=rccl;"
bash scripts/gpu_pass.sh
