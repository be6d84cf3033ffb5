"""Loader for the in-tree gfx950 HIP kernel extension (``_kernels*.so``).

On a GPU the HIP path is mandatory: if the extension is missing or stale this raises
loudly instead of silently falling back to PyTorch ops.  ``INTML_AUTOBUILD=1`` (default)
builds it in-tree on first use when hipcc is available.
"""
from __future__ import annotations

import importlib
import os

_K = None


def kernels():
    global _K
    if _K is not None:
        return _K
    try:
        _K = importlib.import_module("cori_intml_examples_amd._kernels")
    except ImportError as first:
        if os.environ.get("INTML_AUTOBUILD", "1") not in ("0", "false"):
            from .. import _build
            _build.build_kernels()
            importlib.invalidate_caches()
            _K = importlib.import_module("cori_intml_examples_amd._kernels")
        else:
            raise RuntimeError(
                "gfx950 kernel extension not built: run `python -m cori_intml_examples_amd._build` "
                "(HIP path is required on GPU; no PyTorch fallback)") from first
    return _K


def stream_handle(stream=None) -> int:
    import torch
    s = stream or torch.cuda.current_stream()
    return int(s.cuda_stream)
