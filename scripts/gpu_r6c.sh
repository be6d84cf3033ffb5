#!/bin/bash
# round 6: size-1 xGMI admission + the split exchange's forced-structure A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python scripts/probes/xgmi_selftest_p1.py > gpurun_out/r6c_selftest.txt 2>&1 || { cat gpurun_out/r6c_selftest.txt; exit 1; }
cat gpurun_out/r6c_selftest.txt | grep -v amdgpu.ids
export TESTS="tests/test_comm.py" TAG=r6c TESTS_CONTINUE=1 AB_ROUNDS=${AB_ROUNDS:-3} AB_STEPS=600
export AB="|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xchg_p1=1|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xchg_p1=1,xchg_split=0|INTML_DP_FORCE=1 INTML_XGMI=xgmi;|INTML_DP_FORCE=1 INTML_XGMI=rccl;"
bash scripts/gpu_pass.sh
