#!/bin/bash
# Start a one-node farm: one controller + one engine per MI355X (HIP_VISIBLE_DEVICES pinned).
# The cluster id defaults to intml_${SLURM_JOB_ID} under SLURM, else intml_$USER; notebooks
# connect with Client(cluster_id=...).  Extra flags pass through (-n, --gpus, --cpu, --log-file).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export PYTHONPATH="$HERE/..${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python -m cori_intml_examples_amd.farm.cluster start --daemon "$@"
