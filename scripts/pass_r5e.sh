# pass r5e: specialised stack (12 / 16 waves), production kernels, xGMI fence forms at N=1
export TAG=r5e TESTS_CONTINUE=1
export TESTS="tests/test_hip_model.py tests/test_comm.py -k 'specialised or dual_launch or dgrad_onebatch or xgmi or comm'"
export AB="|stack_spec=2|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xgmi_fence=3|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xgmi_fence=0|INTML_DP_FORCE=1 INTML_XGMI=rccl;"
export AB_ROUNDS=2 PROF=rpv PROF_ENV="INTML_TUNE=stack_spec=2"
bash scripts/gpu_pass.sh
