"""Multi-GPU shard loading + RCCL fan-out over xGMI.

The reference is single-GPU (one device picked by index in
utils/nvme_test.c:800-832).  The MI355X design scales the way the node is
built: one process per GPU, each with its own engine instance, NUMA-pinned
I/O workers and its own shard (ideally its own NVMe); loaded shards are then
fanned out with RCCL collectives on a side HIP stream while the next window
is already being read (PAR3 + PAR6):

    step i:   engine loads window i of shard r  ──► HBM buffer[i % 2]
              side stream: all_gather(buffer[(i-1) % 2])  (overlaps the load)
    host:     waits the gather of i-1 before step i+1 reuses that buffer

xGMI is point-to-point (7 links x ~153 GB/s per GPU); a ring all-gather
moves (N-1)/N of the output per rank through one link at a time, which is
still an order of magnitude above one PCIe Gen5 x16 ingest link, so fan-out
hides behind the storage read.  ``mode="broadcast"`` replicates one rank's
window instead (e.g. a shared dimension table).

On CPU (tests) the same code runs with gloo and host-emulated "HBM".
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import api
from ..models.ssd2gpu_stream import StreamLoader
from ..tensor import HbmBuffer


def init_distributed(backend: Optional[str] = None) -> tuple[int, int, torch.device]:
    """Initialise one-process-per-GPU from torchrun's env (127.0.0.1 default)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        be = backend or "nccl"
    else:
        dev = torch.device("cpu")
        be = backend or "gloo"
    if world > 1 and not dist.is_initialized():
        if be == "nccl":
            dist.init_process_group(be, device_id=dev)
        else:
            dist.init_process_group(be)
    return rank, world, dev


def shard_range(total: int, world: int, rank: int, align: int = 1 << 20) -> tuple[int, int]:
    """Contiguous, ``align``-aligned byte range of a file for ``rank``."""
    per = (total + world - 1) // world
    per = (per + align - 1) // align * align
    lo = min(total, rank * per)
    return lo, min(total, lo + per) - lo


class ShardLoadError(RuntimeError):
    """A rank's window load failed; raised on EVERY rank of the group (the
    others would otherwise block in the next collective forever)."""

    def __init__(self, step: int, failed: List[int], cause: Optional[BaseException] = None):
        super().__init__(f"step {step}: window load failed on rank(s) {failed}"
                         + (f": {cause}" if cause else ""))
        self.step = step
        self.failed = failed
        self.cause = cause


@dataclass
class FanoutStats:
    steps: int = 0
    load_s: float = 0.0
    bytes_loaded: int = 0
    bytes_gathered: int = 0
    wall_s: float = 0.0
    windows: List[float] = field(default_factory=list)


class ShardedLoader:
    """Per-rank window loader with collective fan-out of each loaded window."""

    def __init__(self, path: str, window: int, device: torch.device, mode: str = "allgather",
                 src_rank: int = 0, segment_sz: int = 32 << 20, chunk_sz: int = 8192,
                 depth: int = 6, file_offset: int = 0, file_bytes: Optional[int] = None,
                 group=None):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.group = group
        self.mode = mode
        self.src_rank = src_rank
        self.device = device
        self.window = window
        self.file_offset = file_offset
        size = os.path.getsize(path)
        self.file_bytes = file_bytes if file_bytes is not None else size - file_offset
        self.nwin = max(1, self.file_bytes // window)
        self.bufs = [HbmBuffer(window, device) for _ in range(2)]
        segment_sz = min(segment_sz, window)
        self.loader = StreamLoader(path, segment_sz=segment_sz, chunk_sz=chunk_sz,
                                   buf=self.bufs[0], depth=depth)
        self.cuda = device.type == "cuda"
        self.side = torch.cuda.Stream(device=device) if self.cuda else None
        n_out = self.world * window if mode == "allgather" else window
        self.out = torch.empty(n_out, dtype=torch.uint8, device=device) if self.world > 1 else None
        self._pending = None
        self.stats = FanoutStats()

    def _fan(self, buf: torch.Tensor):
        if self.world == 1:
            return None
        if self.mode == "allgather":
            op = lambda: dist.all_gather_into_tensor(self.out, buf, group=self.group, async_op=True)
        else:
            def op():
                if self.rank == self.src_rank:
                    self.out.copy_(buf)
                return dist.broadcast(self.out, self.src_rank, group=self.group, async_op=True)
        if not self.cuda:
            return op()              # gloo: async work handle
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            h = op()
            h.wait()
            done = torch.cuda.Event()
            done.record(self.side)
        return done

    @staticmethod
    def _finish(h) -> None:
        if h is None:
            return
        if isinstance(h, torch.cuda.Event):
            h.synchronize()
        else:
            h.wait()

    def step(self, i: int) -> None:
        buf = self.bufs[i % 2]
        off = self.file_offset + (i % self.nwin) * self.window
        t0 = time.perf_counter()
        err = None
        try:
            st = self.loader.run(off, self.window, buf=buf)
        except (api.StromError, OSError) as e:
            err = e
        self.stats.load_s += time.perf_counter() - t0
        self._agree(i, err)
        self.stats.bytes_loaded += st.bytes
        h = self._fan(buf.tensor)
        # the fan-out of step i-1 overlapped this load; retire it before the
        # next step reuses its buffer
        self._finish(self._pending)
        self._pending = h
        self.stats.steps += 1
        if self.world > 1:
            self.stats.bytes_gathered += self.out.numel()

    def _agree(self, i: int, err: Optional[BaseException]) -> None:
        """Failure consensus before the collective: one 4-byte all-gather of
        per-rank status (RCCL on the GPU), so a read error on one rank
        surfaces as ShardLoadError on all of them instead of a hang."""
        if self.world == 1:
            if err is not None:
                raise ShardLoadError(i, [self.rank], err)
            return
        mine = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=self.device)
        every = torch.empty(self.world, dtype=torch.int32, device=self.device)
        dist.all_gather_into_tensor(every, mine, group=self.group)
        failed = [r for r, v in enumerate(every.tolist()) if v]
        if failed:
            self._finish(self._pending)
            self._pending = None
            raise ShardLoadError(i, failed, err)

    def run(self, steps: int, start: int = 0) -> FanoutStats:
        t0 = time.perf_counter()
        for i in range(start, start + steps):
            self.step(i)
        self.flush()
        self.stats.wall_s += time.perf_counter() - t0
        return self.stats

    def flush(self) -> None:
        self._finish(self._pending)
        self._pending = None
        if self.cuda:
            torch.cuda.current_stream().synchronize()

    def current(self, i: int) -> torch.Tensor:
        return self.bufs[i % 2].tensor

    def close(self) -> None:
        self.flush()
        self.loader.close()
        for b in self.bufs:
            b.close()
