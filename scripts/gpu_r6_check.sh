#!/bin/bash
# round 6: last sanity pass on the in-tree build at the final commit (smoke, driver command,
# the legacy / kernel numerics)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TAG=r6h SMOKE=1 DRIVER=1
export TESTS="tests/test_hip_kernels.py -k 'legacy or bench'"
bash scripts/gpu_pass.sh || exit 1
