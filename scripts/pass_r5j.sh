# pass r5j: the exchange self-test in the xGMI setup, the auto plane, and the DP workflows on
# the GPU (comm / integration / convergence / hpo)
export TAG=r5j TESTS_CONTINUE=1
export TESTS="tests/test_comm.py tests/test_gpu_integration.py tests/test_convergence.py tests/test_hpo.py -m gpu"
bash scripts/gpu_pass.sh
