"""Per-rank I/O placement for one-process-per-GPU jobs.

The engine's reader pool (``workers`` threads, each ``queue_depth`` deep) is
sized for ONE backing device.  When several ranks of a node read from the
same device (a shared array, or the pool box's single filesystem) their
pools add up and the device thrashes: 8 ranks x 4 workers gave 12.7 GiB/s on
the pool box where 8 x 1 gave 21.7 (profiles/r1k).  With one SSD per GPU
(the target layout) every rank keeps the full pool.

So the pool is split by the number of ranks that share THIS rank's backing
device, found by all-gathering (host, device identity) over the job's
process group — the identity is the disk CHECK_FILE classifies the shard
onto (``nvme3n1``, ``md0``), or the filesystem's st_dev for a virtual one.
The same call reports the shard's PCIe affinity to the rank's GPU
(utils/topology.py).
"""
from __future__ import annotations

import os
import socket
from typing import Optional

import torch.distributed as dist

from .. import api
from ..utils import topology


def device_identity(path: str) -> tuple[str, dict]:
    topo = topology.file_topology(path)
    ident = topo["disk"] or f"dev{topo['dev']}"
    return f"{socket.gethostname()}:{ident}", topo


def plan_io(path: str, base_workers: int = 4, device: Optional[int] = None,
            group=None, apply: bool = True) -> dict:
    """Size this rank's reader pool by how many ranks share its device.

    Collective over ``group`` when torch.distributed is initialised (every
    rank must call it); ``apply`` reconfigures the engine."""
    ident, topo = device_identity(path)
    idents = [ident]
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        idents = [None] * dist.get_world_size(group)
        dist.all_gather_object(idents, ident, group=group)
    sharers = idents.count(ident)
    workers = max(1, base_workers // sharers)
    env = os.environ.get("STROM_WORKERS")
    if env:                                   # an explicit setting wins
        workers = int(env)
    aff = None
    if device is not None:
        try:
            aff = topology.file_affinity(path, device)["affinity"]
        except OSError:
            aff = "unknown"
    if apply and str(workers) != api.config_get("workers"):
        api.configure(workers=workers)
    return dict(device=ident.split(":", 1)[1], fs=topo["fs"], sharers=sharers, workers=workers,
                distinct_devices=len(set(idents)), gpu_affinity=aff,
                members=[m["disk"] for m in topo["members"]])
