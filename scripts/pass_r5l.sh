# pass r5l: the whole GPU suite, smoke, the driver's command and kernel stats at the current commit
export TAG=r5l TESTS_CONTINUE=1 TESTS_LIMIT=1100
export TESTS=all SMOKE=1 DRIVER=1 PROF="rpv mnist"
bash scripts/gpu_pass.sh
