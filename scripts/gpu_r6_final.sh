#!/bin/bash
# Round-6 evidence pass at the final kernels: the whole GPU suite, smoke, the driver's exact
# bench command (+ its default N=1 line), the DP step with the N > 1 exchange structure forced,
# B=1024, MNIST and legacy lines, and per-kernel sequences of the three models -- every GPU step
# under its own time limit, stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
O=gpurun_out/${TAG:-r6f}
$T 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > ${O}_tests.log 2>&1
rc=$?; grep -E "passed|failed" ${O}_tests.log | tail -n 2
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR" ${O}_tests.log | head -n 20; exit $rc; fi
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 || { tail -n 20 ${O}_smoke.log; exit 1; }
tail -n 1 ${O}_smoke.log
$T 400 python bench.py --gpus 1 --steps 20 --warmup 5 > ${O}_driver.log 2>&1 || { tail -n 30 ${O}_driver.log; exit 1; }
tail -n 1 ${O}_driver.log | cut -c1-400
$T 400 python bench.py --gpus 1 --steps 20 --warmup 5 > ${O}_driver2.log 2>&1 || { tail -n 30 ${O}_driver2.log; exit 1; }
tail -n 1 ${O}_driver2.log | cut -c1-400
$T 300 python bench.py --steps 600 --warmup 80 --no-hpo --no-dp-delta > ${O}_rpv600.log 2>&1 || { tail -n 30 ${O}_rpv600.log; exit 1; }
tail -n 1 ${O}_rpv600.log | cut -c1-300
INTML_DP_FORCE=1 INTML_XGMI=xgmi INTML_TUNE=xchg_p1=1 $T 300 python bench.py --steps 600 --warmup 80 --no-hpo --no-dp-delta > ${O}_xchg.log 2>&1 || { tail -n 30 ${O}_xchg.log; exit 1; }
tail -n 1 ${O}_xchg.log | cut -c1-300
$T 300 python bench.py --batch 1024 --steps 100 --warmup 20 --no-hpo --no-dp-delta > ${O}_b1024.log 2>&1 || { tail -n 30 ${O}_b1024.log; exit 1; }
tail -n 1 ${O}_b1024.log | cut -c1-300
$T 300 python bench.py --model mnist --steps 600 --warmup 80 --no-hpo --no-dp-delta > ${O}_mnist.log 2>&1 || { tail -n 30 ${O}_mnist.log; exit 1; }
tail -n 1 ${O}_mnist.log | cut -c1-300
$T 300 python bench.py --model rpv_legacy --steps 150 --warmup 20 --no-hpo --no-dp-delta > ${O}_legacy.log 2>&1 || { tail -n 30 ${O}_legacy.log; exit 1; }
tail -n 1 ${O}_legacy.log | cut -c1-300
for m in rpv mnist rpv_legacy; do
  MODEL=$m STEPS=20 WARMUP=5 BENCH_ARGS="--no-hpo --no-dp-delta" bash scripts/prof_model.sh > ${O}_${m}_stats.txt || exit 1
  python scripts/prof_sequence.py gpurun_out/prof_$m/run_kernel_trace.csv > ${O}_${m}_sequence.txt
  cat ${O}_${m}_sequence.txt
done
echo "pass r6f done"
