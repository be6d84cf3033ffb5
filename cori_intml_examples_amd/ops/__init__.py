"""Ops: CPU fp32 reference implementations (``reference``) and the gfx950 HIP kernels
(``hip``, loaded from the in-tree ``_kernels`` extension)."""
from . import reference, rng
