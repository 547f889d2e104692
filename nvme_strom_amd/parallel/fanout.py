"""Multi-GPU shard loading + RCCL fan-out over xGMI.

The reference is single-GPU (one device picked by index in
utils/nvme_test.c:800-832).  The MI355X design scales the way the node is
built: one process per GPU, each with its own engine instance, NUMA-pinned
I/O workers and its own shard (ideally its own NVMe); loaded shards are then
fanned out with RCCL collectives on a side HIP stream while the next window
is already being read (PAR3 + PAR6):

    step i:   engine loads window i of shard r  ──► HBM buffer[i % 2]
              side stream: status word + all_gather(buffer[i % 2])
                           (runs while step i+1 loads the other buffer)
    host:     retires the gather of i-1 before step i+1 reuses that buffer

xGMI is point-to-point (7 links x ~153 GB/s per GPU); a ring all-gather
moves (N-1)/N of the output per rank through one link at a time, which is
still an order of magnitude above one PCIe Gen5 x16 ingest link, so fan-out
hides behind the storage read.  ``mode="broadcast"`` replicates one rank's
window instead (e.g. a shared dimension table).

Failure consensus without a per-step host sync: every step each rank puts a
4-byte status word (0, or step+1 when its load failed) through a tiny
all-gather on the same side stream as the data collective, and the device
keeps, per rank, the first failed step.  The host reads that accumulator
only every ``check_every`` steps and in ``flush()``; since all ranks run the
same collective schedule (a failed rank still joins the data gather, with
its window flagged), every rank raises the same ``ShardLoadError`` at the
same point and none is left blocked in a collective.

``verify(i)`` is the end-to-end integrity check of a fan-out: each rank's
host CRC32C of the file window it loaded at step i is all-gathered and
compared with the CRC of the matching slice of the gathered tensor (on the
GPU for device tensors); the verdict is reduced with MIN so every rank
returns the same bool.

On CPU (tests) the same code runs with gloo and host-emulated "HBM".  With
gloo and device tensors (rehearsing several ranks on one GPU) the
collectives are staged through host memory.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
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


def crc32c_of(t: torch.Tensor) -> int:
    """CRC32C of a uint8 tensor: the CDNA4 kernel for device tensors, the
    engine's host CRC for CPU (gpu_emulation) tensors."""
    if t.is_cuda:
        from ..ops import verify as V
        return V.crc32c(t)
    return api.crc32c_host(t.contiguous().numpy().tobytes())


def file_crc32c(path: str, offset: int, nbytes: int) -> int:
    """Host CRC32C of ``nbytes`` of a file from ``offset`` (zero-padded past EOF,
    like a loaded chunk)."""
    crc, left = 0, nbytes
    with open(path, "rb") as f:
        f.seek(offset)
        while left:
            blk = f.read(min(64 << 20, left)) or b"\0" * left
            crc = api.crc32c_host(blk, crc)
            left -= len(blk)
    return crc


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
    nr_ram: int = 0
    nr_ssd: int = 0
    nr_submit: int = 0
    nr_blocks: int = 0


class ShardedLoader:
    """Per-rank window loader with collective fan-out of each loaded window.

    ``on_loaded(step, window_tensor)`` runs after a window landed and before
    it is fanned out (a consumer hook; tests use it to corrupt a slice)."""

    def __init__(self, path: str, window: int, device: torch.device, mode: str = "allgather",
                 src_rank: int = 0, segment_sz: int = 32 << 20, chunk_sz: int = 8192,
                 depth: int = 6, file_offset: int = 0, file_bytes: Optional[int] = None,
                 group=None, check_every: int = 8,
                 on_loaded: Optional[Callable[[int, torch.Tensor], None]] = None):
        if mode not in ("allgather", "broadcast", "none"):
            raise ValueError(f"mode {mode!r}")
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.group = group
        self.mode = mode
        self.src_rank = src_rank
        self.device = device
        self.path = path
        self.window = window
        self.file_offset = file_offset
        size = os.path.getsize(path)
        self.file_bytes = file_bytes if file_bytes is not None else size - file_offset
        self.nwin = max(1, self.file_bytes // window)
        self.check_every = max(1, int(check_every))
        self.on_loaded = on_loaded
        self.cuda = device.type == "cuda"
        self.fan = self.world > 1 and mode != "none"
        nbuf = 2 if self.fan else 1
        self.bufs = [HbmBuffer(window, device) for _ in range(nbuf)]
        segment_sz = min(segment_sz, window)
        self.loader = StreamLoader(path, segment_sz=segment_sz, chunk_sz=chunk_sz,
                                   buf=self.bufs[0], depth=depth)
        backend = dist.get_backend(group) if self.world > 1 else None
        # gloo cannot run collectives on device memory: stage through the host
        self.staged = self.cuda and backend == "gloo"
        self.side = torch.cuda.Stream(device=device) if self.cuda and not self.staged else None
        cdev = device if (self.cuda and not self.staged) else torch.device("cpu")
        self._cdev = cdev
        n_out = self.world * window if mode == "allgather" else window
        self.out = torch.empty(n_out, dtype=torch.uint8, device=device) if self.fan else None
        # failure consensus words (see module docstring)
        self._status = torch.zeros(1, dtype=torch.int64, device=cdev)
        self._status_all = torch.zeros(self.world, dtype=torch.int64, device=cdev)
        self._first_fail = torch.zeros(self.world, dtype=torch.int64, device=cdev)
        self._local_err: Optional[BaseException] = None
        self._since_check = 0
        self._pending = None
        self._gather_ev: List[tuple] = []        # (start, end) device events
        self.gather_s = 0.0                      # host-timed collectives (CPU/staged)
        self.last_step: Optional[int] = None
        self.stats = FanoutStats()

    # ---- collectives -------------------------------------------------------
    def _collectives(self, buf: torch.Tensor, status: int) -> None:
        """Status word + data collective of one step (issued in this order on
        every rank)."""
        self._status.fill_(status)
        dist.all_gather_into_tensor(self._status_all, self._status, group=self.group)
        self._first_fail.copy_(torch.where(self._first_fail == 0, self._status_all,
                                           self._first_fail))
        if not self.fan:
            return
        if self.mode == "allgather":
            dist.all_gather_into_tensor(self.out, buf, group=self.group)
        else:
            if self.rank == self.src_rank:
                self.out.copy_(buf)
            dist.broadcast(self.out, self.src_rank, group=self.group)

    def _fan(self, buf: torch.Tensor, status: int):
        if self.world == 1:
            return None
        if self.side is None:
            t0 = time.perf_counter()
            if self.staged:
                hbuf = buf.cpu()
                hout = torch.empty(self.out.numel(), dtype=torch.uint8) if self.fan else None
                real_out, self.out = self.out, hout
                try:
                    self._collectives(hbuf, status)
                finally:
                    self.out = real_out
                if self.fan:
                    self.out.copy_(hout)
            else:
                self._collectives(buf, status)
            self.gather_s += time.perf_counter() - t0
            return None
        ev = torch.cuda.Event()
        ev.record()
        start = torch.cuda.Event(enable_timing=True)
        done = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            start.record(self.side)
            self._collectives(buf, status)
            done.record(self.side)
        self._gather_ev.append((start, done))
        return done

    @staticmethod
    def _finish(h) -> None:
        if h is not None:
            h.synchronize()

    # ---- steps -------------------------------------------------------------
    def window_offset(self, i: int) -> int:
        return self.file_offset + (i % self.nwin) * self.window

    def step(self, i: int) -> None:
        buf = self.bufs[i % len(self.bufs)]
        if len(self.bufs) == 1:
            self._finish(self._pending)          # single buffer: gather must be done
            self._pending = None
        t0 = time.perf_counter()
        err = None
        try:
            st = self.loader.run(self.window_offset(i), self.window, buf=buf)
            for k in ("nr_ram", "nr_ssd", "nr_submit", "nr_blocks"):
                setattr(self.stats, k, getattr(self.stats, k) + getattr(st, k))
        except (api.StromError, OSError) as e:
            err = e
            if self._local_err is None:
                self._local_err = e
        self.stats.load_s += time.perf_counter() - t0
        if err is None and self.on_loaded is not None:
            self.on_loaded(i, buf.tensor)
        if err is not None and self.world == 1:
            raise ShardLoadError(i, [self.rank], err)
        h = self._fan(buf.tensor, 0 if err is None else i + 1)
        # the fan-out of step i-1 overlapped this load; retire it before the
        # next step reuses its buffer
        self._finish(self._pending)
        self._pending = h
        self.last_step = i
        self.stats.steps += 1
        if err is None:
            self.stats.bytes_loaded += self.window
        if self.fan:
            self.stats.bytes_gathered += self.out.numel()
        self._since_check += 1
        if self._since_check >= self.check_every:
            self.check()

    def check(self) -> None:
        """Raise ShardLoadError on every rank if any rank failed a load since
        the last check (one host read of the device accumulator)."""
        self._since_check = 0
        if self.world == 1:
            return
        if self.side is not None:
            self.side.synchronize()
        first = self._first_fail.cpu().tolist()
        failed = [r for r, v in enumerate(first) if v]
        if failed:
            self._first_fail.zero_()
            cause, self._local_err = self._local_err, None
            raise ShardLoadError(min(first[r] for r in failed) - 1, failed, cause)

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
        self.check()

    def current(self, i: int) -> torch.Tensor:
        return self.bufs[i % len(self.bufs)].tensor

    # ---- integrity + reporting --------------------------------------------
    def _gather_row(self, vals: List[float], dtype=torch.float64) -> torch.Tensor:
        t = torch.tensor(vals, dtype=dtype, device=self._cdev)
        if self.world == 1:
            return t.reshape(1, -1).cpu()
        out = torch.empty(self.world * t.numel(), dtype=dtype, device=self._cdev)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out.reshape(self.world, -1).cpu()

    def verify(self, i: Optional[int] = None) -> bool:
        """CRC32C of every slice of the fanned-out window of step ``i``
        (default: the last step) against each source rank's host CRC of the
        file window it loaded.  Collective; same verdict on every rank."""
        self.flush()
        i = self.last_step if i is None else i
        mine = file_crc32c(self.path, self.window_offset(i), self.window)
        want = self._gather_row([mine], dtype=torch.int64)[:, 0].tolist()
        if not self.fan:
            ok = crc32c_of(self.bufs[i % len(self.bufs)].tensor) == mine
        elif self.mode == "allgather":
            W = self.window
            ok = all(crc32c_of(self.out[r * W:(r + 1) * W]) == want[r] for r in range(self.world))
        else:
            ok = crc32c_of(self.out) == want[self.src_rank]
        if self.world == 1:
            return ok
        v = torch.tensor([1 if ok else 0], dtype=torch.int64, device=self._cdev)
        dist.all_reduce(v, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(v.item()) == 1)

    def gather_seconds(self) -> float:
        """Summed device time of this rank's step collectives."""
        if self._gather_ev:
            self.side.synchronize()
            s = sum(a.elapsed_time(b) for a, b in self._gather_ev) / 1e3
            self._gather_ev.clear()
            self.gather_s += s
        return self.gather_s

    def report(self, wall_s: Optional[float] = None) -> dict:
        """Per-rank load rate, collective time and load/collective overlap
        (collective).  ``overlap`` is the fraction of collective time hidden
        behind loads: (load + gather - wall) / gather, clamped to [0, 1]."""
        wall = self.stats.wall_s if wall_s is None else wall_s
        g = self.gather_seconds()
        row = [self.stats.bytes_loaded / max(self.stats.load_s, 1e-12) / (1 << 30),
               g * 1e3, self.stats.load_s, wall]
        allr = self._gather_row(row)
        per_gibps = [round(float(x), 3) for x in allr[:, 0].tolist()]
        per_ms = [round(float(x), 3) for x in allr[:, 1].tolist()]
        overlap = []
        for load_s, gms, w in zip(allr[:, 2].tolist(), allr[:, 1].tolist(), allr[:, 3].tolist()):
            gs = gms / 1e3
            overlap.append(round(min(1.0, max(0.0, (load_s + gs - w) / gs)), 3) if gs > 0 else None)
        return {"load_GiBps_per_rank": per_gibps, "collective_ms_per_rank": per_ms,
                "overlap_per_rank": overlap, "steps": self.stats.steps,
                "bytes_gathered_per_rank": self.stats.bytes_gathered}

    def close(self) -> None:
        self._finish(self._pending)
        self._pending = None
        self.loader.close()
        for b in self.bufs:
            b.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
