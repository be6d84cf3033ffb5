# pass r5n: float4 slab reduction for every identity-layout descriptor (conv weights, biases; any
# slab count, 2 split-lanes from 16 slabs) -- model / kernel tests, the three models' lines and
# the legacy kernel stats
export TAG=r5n TESTS_CONTINUE=1
export TESTS="tests/test_hip_kernels.py tests/test_hip_model.py tests/test_comm.py -m gpu -k 'not processes'"
export AB="" AB_ROUNDS=1 AB_STEPS=600
export PROF="rpv_legacy rpv"
bash scripts/gpu_pass.sh && \
for m in mnist rpv_legacy; do timeout -k 10 300 python bench.py --model $m --steps 200 --warmup 20 --no-hpo --no-dp-delta > gpurun_out/r5n_$m.log 2>&1 && tail -c 400 gpurun_out/r5n_$m.log | tr ',' '\n' | grep -E '"value"|ms_per_step' ; done
