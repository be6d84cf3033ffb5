#!/bin/bash
# Images/sec of the headline RPV training step at 1/2/4/8 MI355X on one node (weak scaling,
# batch 128 per GPU), one JSON line per N.  MODEL=mnist|rpv|rpv_legacy selects the config.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODEL=${MODEL:-rpv}
for N in ${GPUS:-1 2 4 8}; do
  if [ "$N" = 1 ]; then
    timeout -k 10 600 python "$HERE/bench.py" --model "$MODEL" --steps ${STEPS:-200} --warmup ${WARMUP:-30} || exit $?
  else
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
      --master-addr 127.0.0.1 --master-port $((29500 + N)) \
      "$HERE/bench.py" --gpus "$N" --model "$MODEL" --steps ${STEPS:-200} --warmup ${WARMUP:-30} || exit $?
  fi
done
