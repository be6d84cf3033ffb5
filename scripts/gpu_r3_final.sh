#!/bin/bash
# Round-3 evidence pass: whole GPU suite, smoke, the default bench (with its HPO record), the
# DP path at N=1, MNIST / legacy benches, RPV kernel stats and PMC -- every GPU step under its
# own time limit, stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 6 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -n 20 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
$T 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -n 30 gpurun_out/bench_default.log; exit 1; }
tail -n 1 gpurun_out/bench_default.log | cut -c1-300
INTML_DP_FORCE=1 $T 300 python bench.py --steps 400 --warmup 40 --no-hpo > gpurun_out/bench_dp1.log 2>&1 || { tail -n 30 gpurun_out/bench_dp1.log; exit 1; }
tail -n 1 gpurun_out/bench_dp1.log | cut -c1-200
$T 300 python bench.py --model mnist --steps 400 --warmup 40 --no-hpo > gpurun_out/bench_mnist.log 2>&1 || { tail -n 30 gpurun_out/bench_mnist.log; exit 1; }
tail -n 1 gpurun_out/bench_mnist.log | cut -c1-200
$T 300 python bench.py --model rpv_legacy --steps 40 --warmup 10 --no-hpo > gpurun_out/bench_legacy.log 2>&1 || { tail -n 30 gpurun_out/bench_legacy.log; exit 1; }
tail -n 1 gpurun_out/bench_legacy.log | cut -c1-200
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/prof_rpv_summary.txt || exit 1
head -14 gpurun_out/prof_rpv_summary.txt
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc1 -o run -- python $R/bench.py --steps 16 --warmup 8 --no-hpo > $R/gpurun_out/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -n 5 $R/gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmc2 -o run -- python $R/bench.py --steps 16 --warmup 8 --no-hpo > $R/gpurun_out/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -n 5 $R/gpurun_out/pmc2.log; exit 1; }
cd $R && python scripts/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv gpurun_out/pmc2/run_counter_collection.csv > gpurun_out/pmc_summary.txt 2>&1; grep -- "->" gpurun_out/pmc_summary.txt | head -20
