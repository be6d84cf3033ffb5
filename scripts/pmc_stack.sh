#!/bin/bash
# PMC counters of the layer-fused conv-stack kernel (one rocprofv3 pass per counter set).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc1 -o run -- python $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -n 20 $R/gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_ADDR_CONFLICT --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc2 -o run -- python $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -n 20 $R/gpurun_out/pmc2.log; exit 1; }
ls $R/gpurun_out/pmc1 $R/gpurun_out/pmc2
