#!/bin/bash
# Evidence pass (via gpurun): rocprofv3 kernel stats of the RPV bench step, two PMC passes
# (instruction mix / LDS conflicts / waits) and an HBM-bytes pass, summarised into
# gpurun_out/${TAG}_*.txt.  Each profiler run has its own time limit; stops at the first failure.
set -e -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-v11}
cd $R && mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- \
    python $R/bench.py --steps 24 --warmup 8 > $R/gpurun_out/${TAG}_prof.log 2>&1
cd $R && python scripts/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv 32 > gpurun_out/${TAG}_rpv_kernel_stats.txt
head -n 14 gpurun_out/${TAG}_rpv_kernel_stats.txt
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_BUSY_CYCLES \
    --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc1 -o run -- python $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/${TAG}_pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM \
    --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc2 -o run -- python $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/${TAG}_pmc2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE \
    --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc3 -o run -- python $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/${TAG}_pmc3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE \
    --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc4 -o run -- python $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/${TAG}_pmc4.log 2>&1
cd $R && python scripts/pmc_summary.py gpurun_out/${TAG}_pmc1/run_counter_collection.csv gpurun_out/${TAG}_pmc2/run_counter_collection.csv \
    gpurun_out/${TAG}_pmc3/run_counter_collection.csv gpurun_out/${TAG}_pmc4/run_counter_collection.csv > gpurun_out/${TAG}_pmc.txt
grep -- "->" gpurun_out/${TAG}_pmc.txt | head -n 20
