# pass r5m: legacy RPV (34.5M) kernel stats at the current kernels, and its bench line
export TAG=r5m
export PROF="rpv_legacy" PROF_STEPS=20
export BENCH="--model rpv_legacy --steps 60 --warmup 10 --no-hpo"
bash scripts/gpu_pass.sh
