#!/bin/bash
# PMC passes of one model's bench step (own runs, --kernel-trace only besides the counters):
#   MODEL=rpv_legacy TAG=r3_legacy bash scripts/gpu_pmc.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
MODEL=${MODEL:-rpv}
TAG=${TAG:-r3_$MODEL}
ST=${STEPS:-10}
cd $R && mkdir -p gpurun_out
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_BUSY_CYCLES \
    --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc1 -o run -- python3 $R/bench.py --model $MODEL --steps $ST --warmup 2 --no-hpo > $R/gpurun_out/${TAG}_pmc1.log 2>&1 || { echo "pmc1 failed"; tail -n 5 $R/gpurun_out/${TAG}_pmc1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM \
    --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc2 -o run -- python3 $R/bench.py --model $MODEL --steps $ST --warmup 2 --no-hpo > $R/gpurun_out/${TAG}_pmc2.log 2>&1 || { echo "pmc2 failed"; tail -n 5 $R/gpurun_out/${TAG}_pmc2.log; exit 1; }
cd $R && python scripts/pmc_summary.py gpurun_out/${TAG}_pmc1/run_counter_collection.csv gpurun_out/${TAG}_pmc2/run_counter_collection.csv > gpurun_out/${TAG}_pmc.txt
grep -B1 -- "->" gpurun_out/${TAG}_pmc.txt | head -n 60
