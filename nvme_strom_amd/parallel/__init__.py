"""Multi-GPU: one process per GPU, shard loading + RCCL fan-out over xGMI."""
from .fanout import (FanoutStats, ShardedLoader, ShardLoadError, init_distributed,  # noqa: F401
                     shard_range)
from .placement import device_identity, plan_io  # noqa: F401
from .scan import DistScanOut, DistributedArrowScan, DistributedHeapScan, partition  # noqa: F401
