"""Multi-GPU: one process per GPU, shard loading + RCCL fan-out over xGMI."""
from .fanout import FanoutStats, ShardedLoader, init_distributed, shard_range  # noqa: F401
