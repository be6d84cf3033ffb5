# pass r5f: producer push of the early (head / dense) bucket on the xGMI plane (P = 2/4/8 ranks on
# one GPU), the GPU model / comm / DP tests on the new defaults (16-wave stack), and the planes at N=1
export TAG=r5f TESTS_CONTINUE=1
export TESTS="tests/test_comm.py tests/test_hip_model.py tests/test_gpu_integration.py tests/test_dense_bwd.py"
export AB="|INTML_DP_FORCE=1 INTML_XGMI=xgmi;|INTML_DP_FORCE=1 INTML_XGMI=rccl;|INTML_DP_FORCE=1 INTML_XGMI=rccl INTML_BUCKET_BYTES=1048576;"
export AB_ROUNDS=2
bash scripts/gpu_pass.sh
