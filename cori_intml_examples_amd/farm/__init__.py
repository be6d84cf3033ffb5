"""One-node task farm: controller + one engine per MI355X, IPyParallel-shaped client API.

Replaces IPyParallel/ZeroMQ/SLURM bring-up of the reference (SURVEY.md §2.3 E5/E6/E11,
§2.5 P2 task farm, P3 HPO x DP, P4 SPMD ``%%px``)."""
from .client import AsyncResult, Client, DirectView, LoadBalancedView
from .cluster import Cluster, default_cluster_id, detect_gpus, start_cluster
from .engine import engine_id, engine_namespace, publish_data, should_stop
from .protocol import EngineError, RemoteError, TaskAborted

__all__ = ["Client", "DirectView", "LoadBalancedView", "AsyncResult", "Cluster", "start_cluster",
           "default_cluster_id", "detect_gpus", "publish_data", "should_stop", "engine_id", "engine_namespace", "RemoteError",
           "TaskAborted", "EngineError"]
