# pass r5o: legacy dense (33.5M-weight) forward geometry -- workgroups per launch / k-steps
export TAG=r5o
export AB="|dense_big_wgs=512|dense_big_wgs=1024,dense_big_minks=4|dense_big_wgs=512,dense_big_minks=4"
export AB_MODEL=rpv_legacy AB_STEPS=200 AB_ROUNDS=2
bash scripts/gpu_pass.sh
