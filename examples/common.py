"""Shared helpers for the notebook-workflow scripts: farm bring-up / connection."""
import argparse
import os

import _path  # noqa: F401
from cori_intml_examples_amd import farm


def farm_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    p.add_argument("--cluster-id", default=None, help="connect to this farm (default: start one)")
    p.add_argument("--engines", type=int, default=None, help="engines to start (default: one per GPU)")
    p.add_argument("--cpu", action="store_true", help="CPU-only engines (no GPU on this host)")
    return p


def connect(args):
    """(client, cluster-or-None): connect to ``--cluster-id`` or start a private farm."""
    if args.cluster_id:
        return farm.Client(cluster_id=args.cluster_id, timeout=60), None
    cpu = args.cpu or farm.detect_gpus() == 0
    cl = farm.start_cluster(args.engines or (2 if cpu else None), cluster_id="examples_%d" % os.getpid(),
                            cpu_only=cpu)
    return cl.client(), cl
