#!/bin/bash
# Environment for the MI355X framework (counterpart of the reference's module loads and
# OpenMP/TF thread settings).  Source it: `source setup.sh`.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export PYTHONPATH="$HERE/..${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=0          # dmabuf IPC for RCCL / cross-process tensors
export PYTORCH_ROCM_ARCH=gfx950
# host-side threads (data prep, CPU reference backend); read by mlextras.configure_session
export NUM_INTER_THREADS=${NUM_INTER_THREADS:-2}
export NUM_INTRA_THREADS=${NUM_INTRA_THREADS:-16}
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-$NUM_INTRA_THREADS}
# build the HIP kernels (gfx950) and the HDF5 module in-tree if needed
python -m cori_intml_examples_amd._build >/dev/null
