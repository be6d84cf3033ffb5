#!/bin/bash
# Round-3 iteration pass: numerics first (bisecting the new kernel paths on failure), then the
# whole GPU suite, the 1-GPU bench, kernel stats and the backward timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -q --timeout 180 --timeout-method thread"
$T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py -x > gpurun_out/numerics.log 2>&1
rc=$?
tail -n 25 gpurun_out/numerics.log
if [ $rc -eq 1 ]; then
  for tn in "lds_layout=0"; do
    echo "== bisect INTML_TUNE=$tn"
    INTML_TUNE=$tn $T 600 $PYT tests/test_hip_model.py tests/test_hip_kernels.py -x > gpurun_out/bisect_$tn.log 2>&1
    r=$?; tail -n 3 gpurun_out/bisect_$tn.log
    if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
  done
  exit 1
fi
if [ $rc -ne 0 ]; then exit $rc; fi
$T 900 $PYT tests -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -n 30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
$T 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log
MODEL=rpv bash scripts/prof_model.sh > gpurun_out/prof_rpv_summary.txt || exit 1
head -24 gpurun_out/prof_rpv_summary.txt
$T 120 python scripts/bwd_timeline.py > gpurun_out/bwd_timeline.txt 2>&1; tail -n 30 gpurun_out/bwd_timeline.txt
# PMC passes (own runs, --kernel-trace only besides the counters)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc1 -o run -- python $R/bench.py --steps 16 --warmup 8 --no-hpo > $R/gpurun_out/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -n 5 $R/gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmc2 -o run -- python $R/bench.py --steps 16 --warmup 8 --no-hpo > $R/gpurun_out/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -n 5 $R/gpurun_out/pmc2.log; exit 1; }
cd $R && python scripts/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv gpurun_out/pmc2/run_counter_collection.csv > gpurun_out/pmc_summary.txt 2>&1; grep -- "->" gpurun_out/pmc_summary.txt | head -20
