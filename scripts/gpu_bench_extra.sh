cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --model mnist --steps 100 --warmup 20 > gpurun_out/bench_mnist.log 2>&1; tail -n 1 gpurun_out/bench_mnist.log
timeout -k 10 300 python bench.py --model rpv_legacy --steps 50 --warmup 10 > gpurun_out/bench_legacy.log 2>&1; tail -n 3 gpurun_out/bench_legacy.log
timeout -k 10 300 python bench.py --batch 1024 --steps 100 --warmup 20 > gpurun_out/bench_b1024.log 2>&1; tail -n 1 gpurun_out/bench_b1024.log
timeout -k 10 600 python benchmarks/hpo_throughput.py --trials 16 > gpurun_out/hpo.log 2>&1; tail -n 1 gpurun_out/hpo.log
