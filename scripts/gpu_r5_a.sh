#!/bin/bash
# Round-5 pass A: baseline of this round's box -- GPU suite, the driver's exact bench command,
# the driver-gap probe (repeated 20-step replays in one process; idle / pre-spin variants), and
# a kernel trace of the driver's command without the HPO record.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5a_gpu_tests.log 2>&1
rc=$?; tail -n 4 gpurun_out/r5a_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a_bench_driver.log 2>&1 || { tail -n 30 gpurun_out/r5a_bench_driver.log; exit 1; }
tail -n 1 gpurun_out/r5a_bench_driver.log | cut -c1-400
$T 200 python scripts/driver_gap.py --reps 30 > gpurun_out/r5a_gap.txt 2>&1 || { tail -n 20 gpurun_out/r5a_gap.txt; exit 1; }
tail -n 31 gpurun_out/r5a_gap.txt
$T 200 python scripts/driver_gap.py --reps 10 --idle-ms 200 > gpurun_out/r5a_gap_idle.txt 2>&1 || { tail -n 20 gpurun_out/r5a_gap_idle.txt; exit 1; }
tail -n 11 gpurun_out/r5a_gap_idle.txt
$T 200 python scripts/driver_gap.py --reps 5 --spin-ms 1000 > gpurun_out/r5a_gap_spin.txt 2>&1 || { tail -n 20 gpurun_out/r5a_gap_spin.txt; exit 1; }
tail -n 6 gpurun_out/r5a_gap_spin.txt
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && $T 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5a_trace -o run -- python $R/scripts/driver_gap.py --reps 6 > $R/gpurun_out/r5a_trace.log 2>&1 || { tail -n 20 $R/gpurun_out/r5a_trace.log; exit 1; }
cd $R && tail -n 7 gpurun_out/r5a_trace.log
