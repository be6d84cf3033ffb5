#!/bin/bash
# Non-interactive data-parallel RPV training on one MI355X node: one rank per GPU over RCCL.
#SBATCH -J train-rpv
#SBATCH -N 1
#SBATCH -t 2:00:00
#SBATCH -o logs/%x-%j.out
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
source "$HERE/setup.sh"
NGPUS=${NGPUS:-8}
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPUS" \
    --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29500} \
    "$HERE/train_rpv.py" --lr-scaling linear "$@"
