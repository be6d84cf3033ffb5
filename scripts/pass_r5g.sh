# pass r5g: the early (head / dense) bucket's whole all-reduce + update inside the backward on the
# xGMI plane (exchange, XgmiPush mode 2) -- P = 2/4/8 ranks on one GPU, the model tests, and the
# DP planes at N=1 against non-DP
export TAG=r5g TESTS_CONTINUE=1
export TESTS="tests/test_comm.py tests/test_hip_model.py -k 'xgmi or dual or early or fused'"
export AB="|INTML_DP_FORCE=1 INTML_XGMI=xgmi;|INTML_DP_FORCE=1 INTML_XGMI=xgmi;xgmi_xchg=0"
export AB_ROUNDS=2
bash scripts/gpu_pass.sh
