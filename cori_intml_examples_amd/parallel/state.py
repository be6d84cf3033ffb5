"""Process-level data-parallel state (one process per GPU)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Optional


@dataclass
class DPState:
    rank: int
    size: int
    local_rank: int
    local_size: int
    backend: str
    shard_data: bool = True
    bucket_bytes: Optional[int] = None   # None: adaptive (dist.adaptive_bucket_bytes)
    owns_pg: bool = False
    comm: Any = None              # parallel.comm.NativeComm (RCCL data plane) or None
    xgmi_only: bool = False       # no RCCL communicator: the fused xGMI kernel is the data plane
    plane: Optional[str] = None   # how init chose the data plane (reported on stderr / History)


_STATE: Optional[DPState] = None


def current() -> Optional[DPState]:
    return _STATE


def set_state(s: Optional[DPState]) -> None:
    global _STATE
    _STATE = s
