# pass r5h: the exchange at N = 1 (the range's update moves into dual conv1; the fused kernel keeps
# the conv layers) -- DP xgmi vs non-DP, and a kernel-stats profile of the DP xgmi step
export TAG=r5h
export TESTS="tests/test_comm.py -k 'dp_step_xgmi'"
export AB="|INTML_DP_FORCE=1 INTML_XGMI=xgmi;|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xchg_rfirst=0|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xgmi_xchg=0"
export AB_ROUNDS=2
export PROF=rpv PROF_ENV="INTML_DP_FORCE=1 INTML_XGMI=xgmi"
bash scripts/gpu_pass.sh
