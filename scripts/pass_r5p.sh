# pass r5p: legacy dense forward / dX with weights two stages ahead + XCD-aware block order
export TAG=r5p TESTS_CONTINUE=1
export TESTS="tests/test_dense_bwd.py tests/test_hip_model.py -m gpu -k 'legacy or dense'"
export AB="|dense_big_wgs=128"
export AB_MODEL=rpv_legacy AB_STEPS=200 AB_ROUNDS=2
export PROF=rpv_legacy
bash scripts/gpu_pass.sh
