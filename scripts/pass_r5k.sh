# pass r5k: shared-GPU detection by physical device identity (farm engines pinned to one GPU),
# the size-1 xGMI plane's exchange tables -- the two failures of r5j plus the DP xGMI rehearsal
export TAG=r5k TESTS_CONTINUE=1
export TESTS="tests/test_comm.py tests/test_gpu_integration.py -m gpu -k 'native_comm_engine or px_engines or dp_step_xgmi or xgmi_processes'"
bash scripts/gpu_pass.sh
