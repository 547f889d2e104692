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

Delivery: the gathered outputs are a ring of ``out_ring``
buffers, step i in buffer i % out_ring, so step i's shards stay readable
while steps i+1.. load and gather.  A consumer either

  * registers ``on_gathered(g)``: called once per step, on the host, when
    the step's gather has completed (during the next step's load), with
    the loader's consumer stream current — GPU work it enqueues there is
    ordered after the gather, and the buffer is retired only after it; or
  * pulls: ``g = ld.gathered(i)`` (blocks until step i was issued; another
    thread may call it), ``g.wait(stream)`` orders its stream after the
    gather, ``ld.release(i, stream)`` records when it is done.  A held
    buffer is not gathered into again until it is released: the side
    stream waits on the release event (the host waits for the release
    call itself).

``verify_each`` checks every step's fan-out on the device: each rank's CRC32C
of its window, taken as it lands, travels in the step's status word; after
the gather every receiver CRCs each slice and keeps, per source rank, the
first step whose slice did not match.  ``check()`` all-gathers those (one
small collective per check) and raises ``ShardCorruptError`` on EVERY rank.
``verify(i)`` is the end-to-end check against the FILE: each rank's host
CRC32C of the window it loaded at step i is all-gathered and compared with
the CRC of the matching slice of the gathered tensor; the verdict is
reduced with MIN so every rank returns the same bool.

On CPU (tests) the same code runs with gloo and host-emulated "HBM".  With
gloo and device tensors (rehearsing several ranks on one GPU) the
collectives are staged through host memory.
"""
from __future__ import annotations

import os
import threading
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

    def __init__(self, step: int, failed: List[int], cause: Optional[BaseException] = None,
                 what: str = "window load failed"):
        super().__init__(f"step {step}: {what} on rank(s) {failed}"
                         + (f": {cause}" if cause else ""))
        self.step = step
        self.failed = failed
        self.cause = cause


class ShardCorruptError(ShardLoadError):
    """``verify_each``: a gathered slice did not match its source rank's CRC
    of the window it loaded (``failed`` = the source ranks); raised on every
    rank at the same check."""

    def __init__(self, step: int, failed: List[int]):
        super().__init__(step, failed, what="gathered slice corrupt from")


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
    delivered: int = 0          # steps handed to on_gathered


@dataclass
class Gathered:
    """One step's fanned-out output as a consumer sees it: ``tensor`` is the
    ring buffer holding it (world x window for all-gather, window for
    broadcast), valid once ``event`` (device path) has completed."""
    step: int
    tensor: torch.Tensor
    window: int
    mode: str
    event: Optional[object] = None

    def slice(self, rank: int) -> torch.Tensor:
        """The window source ``rank`` loaded (broadcast: the one window)."""
        if self.mode == "allgather":
            return self.tensor[rank * self.window:(rank + 1) * self.window]
        return self.tensor

    def wait(self, stream=None) -> None:
        """Order ``stream`` (default: the current one) after the gather."""
        if self.event is not None:
            (stream or torch.cuda.current_stream(self.tensor.device)).wait_event(self.event)


class ShardedLoader:
    """Per-rank window loader with collective fan-out of each loaded window.

    ``on_loaded(step, window_tensor)`` runs after a window landed and before
    it is fanned out (a producer hook; tests use it to corrupt a slice).
    ``on_gathered(g: Gathered)`` / ``gathered(i)`` + ``release(i)``: the
    consumer side (module docstring)."""

    def __init__(self, path: str, window: int, device: torch.device, mode: str = "allgather",
                 src_rank: int = 0, segment_sz: int = 32 << 20, chunk_sz: int = 8192,
                 depth: int = 6, file_offset: int = 0, file_bytes: Optional[int] = None,
                 group=None, check_every: int = 8,
                 on_loaded: Optional[Callable[[int, torch.Tensor], None]] = None,
                 out_ring: int = 2, on_gathered: Optional[Callable[[Gathered], None]] = None,
                 verify_each: bool = False, release_timeout: float = 600.0,
                 force_fan: bool = False):
        if mode not in ("allgather", "broadcast", "none"):
            raise ValueError(f"mode {mode!r}")
        if out_ring < 1:
            raise ValueError("out_ring >= 1")
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
        self.on_gathered = on_gathered
        self.cuda = device.type == "cuda"
        # force_fan: collectives even in a one-rank group (a single-GPU box
        # runs the side-stream / RCCL path of the multi-GPU node this way)
        self.fan = (self.world > 1 or (force_fan and dist.is_initialized())) and mode != "none"
        self._solo = self.world == 1 and not self.fan
        self.verify_each = bool(verify_each) and self.fan
        self.release_timeout = release_timeout
        nbuf = 2 if self.fan else 1
        self.bufs = [HbmBuffer(window, device) for _ in range(nbuf)]
        segment_sz = min(segment_sz, window)
        self.loader = StreamLoader(path, segment_sz=segment_sz, chunk_sz=chunk_sz,
                                   buf=self.bufs[0], depth=depth)
        backend = dist.get_backend(group) if not self._solo else None
        # gloo cannot run collectives on device memory: stage through the host
        self.staged = self.cuda and backend == "gloo"
        self.side = torch.cuda.Stream(device=device) if self.cuda and not self.staged else None
        self.consumer = torch.cuda.Stream(device=device) if self.side is not None else None
        cdev = device if (self.cuda and not self.staged) else torch.device("cpu")
        self._cdev = cdev
        n_out = self.world * window if mode == "allgather" else window
        R = out_ring if self.fan else 0
        self.out_ring = R
        self.outs = [torch.empty(n_out, dtype=torch.uint8, device=device) for _ in range(R)]
        self._slot_step = [-1] * R
        self._slot_done: List[Optional[object]] = [None] * R    # gather complete (device)
        self._slot_rel: List[list] = [[] for _ in range(R)]      # consumer releases (device)
        self._held = [False] * R
        self._cv = threading.Condition()
        self._issued = -1
        self._retired = -1
        # failure consensus words (see module docstring): [status] or, with
        # verify_each, [status, crc32c of the window as it landed]
        self._sw = 2 if self.verify_each else 1
        self._status = torch.zeros(self._sw, dtype=torch.int64, device=cdev)
        self._status_all = torch.zeros(self.world * self._sw, dtype=torch.int64, device=cdev)
        self._first_fail = torch.zeros(self.world, dtype=torch.int64, device=cdev)
        self._first_bad = torch.zeros(self.world, dtype=torch.int64, device=cdev)
        # the landed window's CRC per step parity: written on the loading
        # stream, read into the status word on the side stream (the status
        # word itself may still be read by the previous step's collective)
        self._crc_src = (torch.zeros(2, dtype=torch.int32, device=device)
                         if self.cuda and not self.staged else None)
        self._crc_host = [0, 0]
        srcs = list(range(self.world)) if mode == "allgather" else [src_rank]
        self._srcs = srcs
        self._src_idx = torch.tensor(srcs, dtype=torch.long, device=cdev)
        self._local_err: Optional[BaseException] = None
        self._since_check = 0
        self._pending = None
        self._gather_ev: List[tuple] = []        # (start, end) device events
        self._crc_ev: List[tuple] = []
        self.gather_s = 0.0                      # host-timed collectives (CPU/staged)
        self.crc_s = 0.0
        self.last_step: Optional[int] = None
        self.stats = FanoutStats()

    @property
    def out(self) -> Optional[torch.Tensor]:
        """The last issued step's gathered output (None without fan-out)."""
        if not self.fan:
            return None
        return self.outs[(self.last_step or 0) % self.out_ring]

    # ---- integrity on the fly (verify_each) --------------------------------
    def _src_crc(self, buf: torch.Tensor, step: int) -> None:
        """CRC of the window as it landed (device: on the current stream, no
        host read); _collectives puts it in status word 1."""
        if self._crc_src is not None:
            from ..ops.verify import crc32c_into
            crc32c_into(buf, self._crc_src[step % 2:step % 2 + 1])
        else:
            self._crc_host[step % 2] = crc32c_of(buf)

    def _check_slices(self, out: torch.Tensor, sa: torch.Tensor, step: int) -> None:
        """Every slice of this step's output against its source rank's CRC:
        the first mismatching step per source rank stays in _first_bad."""
        W = self.window
        srcs = self._srcs
        if out.is_cuda:
            from ..ops.verify import crc32c_into
            got32 = torch.zeros(len(srcs), dtype=torch.int32, device=out.device)
            for j, r in enumerate(srcs):
                crc32c_into(out[j * W:(j + 1) * W] if self.mode == "allgather" else out, got32[j:j + 1])
            got = got32.to(torch.int64) & 0xFFFFFFFF
        else:
            got = torch.tensor([crc32c_of(out[j * W:(j + 1) * W] if self.mode == "allgather" else out)
                                for j, _ in enumerate(srcs)], dtype=torch.int64)
        got = got.to(sa.device)
        idx = self._src_idx
        want = sa[idx, 1] & 0xFFFFFFFF
        bad = (got != want) & (sa[idx, 0] == 0)        # a failed load is reported as such
        cur = self._first_bad[idx]
        self._first_bad[idx] = torch.where((cur == 0) & bad, torch.full_like(cur, step + 1), cur)

    # ---- collectives -------------------------------------------------------
    def _collectives(self, buf: torch.Tensor, status: int, step: int, out) -> None:
        """Status word(s) + data collective of one step (issued in this order
        on every rank), then the slice check."""
        self._status[0:1].fill_(status)
        if self.verify_each:
            if self._crc_src is not None:
                c = self._crc_src[step % 2:step % 2 + 1]
                self._status[1:2].copy_(c.to(torch.int64) & 0xFFFFFFFF)
            else:
                self._status[1] = self._crc_host[step % 2]
        dist.all_gather_into_tensor(self._status_all, self._status, group=self.group)
        sa = self._status_all.view(self.world, self._sw)
        self._first_fail.copy_(torch.where(self._first_fail == 0, sa[:, 0], self._first_fail))
        if not self.fan:
            return
        if self.mode == "allgather":
            dist.all_gather_into_tensor(out, buf, group=self.group)
        else:
            if self.rank == self.src_rank:
                out.copy_(buf)
            dist.broadcast(out, self.src_rank, group=self.group)
        if self.verify_each:
            if self.side is not None:
                c0 = torch.cuda.Event(enable_timing=True)
                c1 = torch.cuda.Event(enable_timing=True)
                c0.record(self.side)
                self._check_slices(out, sa, step)
                c1.record(self.side)
                self._crc_ev.append((c0, c1))
            else:
                t0 = time.perf_counter()
                self._check_slices(out, sa, step)
                self.crc_s += time.perf_counter() - t0

    def _fan(self, buf: torch.Tensor, status: int, step: int):
        if self._solo:
            return None
        slot = step % self.out_ring if self.fan else 0
        out = self.outs[slot] if self.fan else None
        if self.side is None:
            t0 = time.perf_counter()
            if self.staged:
                hbuf = buf.cpu()
                hout = torch.empty(out.numel(), dtype=torch.uint8) if self.fan else None
                self._collectives(hbuf, status, step, hout)
                if self.fan:
                    out.copy_(hout)
            else:
                self._collectives(buf, status, step, out)
            self.gather_s += time.perf_counter() - t0
            return None
        ev = torch.cuda.Event()
        ev.record()
        start = torch.cuda.Event(enable_timing=True)
        done = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            if self.fan:
                # the consumer's releases of the step this buffer held
                for rel in self._slot_rel[slot]:
                    self.side.wait_event(rel)
                self._slot_rel[slot] = []
            start.record(self.side)
            self._collectives(buf, status, step, out)
            done.record(self.side)
        if self.fan:
            self._slot_done[slot] = done
        self._gather_ev.append((start, done))
        return done

    @staticmethod
    def _finish(h) -> None:
        if h is not None:
            h.synchronize()

    # ---- the consumer side -------------------------------------------------
    def _acquire(self, step: int) -> None:
        """Wait (host) until the ring buffer step ``step`` gathers into is
        no longer held by a consumer."""
        if not self.fan:
            return
        slot = step % self.out_ring
        with self._cv:
            if not self._cv.wait_for(lambda: not self._held[slot], timeout=self.release_timeout):
                raise RuntimeError(f"step {self._slot_step[slot]}'s gathered output was not "
                                   f"released within {self.release_timeout} s (ring of "
                                   f"{self.out_ring})")
            self._slot_step[slot] = step

    def _publish(self, step: int) -> None:
        with self._cv:
            self._issued = step
            self._cv.notify_all()

    def _gathered_obj(self, step: int) -> Gathered:
        slot = step % self.out_ring
        return Gathered(step, self.outs[slot], self.window, self.mode, self._slot_done[slot])

    def _retire(self, upto: int) -> None:
        """Hand every step up to ``upto`` whose gather has completed to
        on_gathered (its GPU work on the consumer stream, after the gather;
        the buffer's release is recorded after it)."""
        while self._retired < upto:
            j = self._retired + 1
            self._retired = j
            if not self.fan or self.on_gathered is None or j < 0:
                continue
            g = self._gathered_obj(j)
            if self.consumer is not None:
                g.wait(self.consumer)
                with torch.cuda.stream(self.consumer):
                    self.on_gathered(g)
                rel = torch.cuda.Event()
                rel.record(self.consumer)
                self._slot_rel[j % self.out_ring].append(rel)
            else:
                self.on_gathered(g)
            self.stats.delivered += 1

    def gathered(self, i: int, timeout: Optional[float] = None) -> Gathered:
        """Step ``i``'s gathered output, held until ``release(i)``: blocks
        until the step was issued (the returned ``event`` orders a stream
        after its gather — ``g.wait(stream)``); LookupError when the ring has
        moved past it."""
        if not self.fan:
            raise RuntimeError("no fan-out (world size 1 or mode 'none'): use current(i)")
        slot = i % self.out_ring
        with self._cv:
            if not self._cv.wait_for(lambda: self._issued >= i, timeout=timeout):
                raise TimeoutError(f"step {i} not gathered within {timeout} s")
            if self._slot_step[slot] != i:
                raise LookupError(f"step {i} left the ring (buffer holds step {self._slot_step[slot]})")
            self._held[slot] = True
            return self._gathered_obj(i)

    def release(self, i: int, stream=None) -> None:
        """The consumer is done with step ``i``'s output (device: once the
        work queued so far on ``stream`` / the current stream completes)."""
        slot = i % self.out_ring
        with self._cv:
            if self._slot_step[slot] != i:
                raise LookupError(f"step {i} is not in the ring")
            if self.side is not None:
                ev = torch.cuda.Event()
                ev.record(stream or torch.cuda.current_stream(self.device))
                self._slot_rel[slot].append(ev)
            self._held[slot] = False
            self._cv.notify_all()

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
        if err is None and self.verify_each:
            self._src_crc(buf.tensor, i)
        if err is None and self.on_loaded is not None:
            self.on_loaded(i, buf.tensor)
        if err is not None and self._solo:
            raise ShardLoadError(i, [self.rank], err)
        self._acquire(i)
        h = self._fan(buf.tensor, 0 if err is None else i + 1, i)
        self._publish(i)
        # the fan-out of step i-1 overlapped this load; retire it (and hand
        # it to the consumer) before the next step reuses its buffer
        self._finish(self._pending)
        self._retire(i - 1 if h is not None else i)
        self._pending = h
        self.last_step = i
        self.stats.steps += 1
        if err is None:
            self.stats.bytes_loaded += self.window
        if self.fan:
            self.stats.bytes_gathered += self.outs[0].numel()
        self._since_check += 1
        if self._since_check >= self.check_every:
            self.check()

    def check(self) -> None:
        """Raise ShardLoadError (a load failed) or ShardCorruptError (a
        gathered slice did not match) on every rank, for anything since the
        last check (one host read of the device accumulators; with
        verify_each one small all-gather of them — collective)."""
        self._since_check = 0
        if self._solo:
            return
        if self.side is not None:
            self.side.synchronize()
        bad = None
        if self.verify_each:
            allb = torch.empty(self.world * self.world, dtype=torch.int64, device=self._cdev)
            dist.all_gather_into_tensor(allb, self._first_bad, group=self.group)
            bad = allb.view(self.world, self.world).cpu()
            self._first_bad.zero_()
        first = self._first_fail.cpu().tolist()
        failed = [r for r, v in enumerate(first) if v]
        if failed:
            self._first_fail.zero_()
            cause, self._local_err = self._local_err, None
            raise ShardLoadError(min(first[r] for r in failed) - 1, failed, cause)
        if bad is not None and bool((bad > 0).any()):
            b = torch.where(bad > 0, bad, torch.full_like(bad, 1 << 62)).min(dim=0).values
            srcs = [r for r in range(self.world) if int(b[r]) < (1 << 62)]
            raise ShardCorruptError(min(int(b[r]) for r in srcs) - 1, srcs)

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
        if self.last_step is not None:
            self._retire(self.last_step)
        if self.cuda:
            torch.cuda.current_stream().synchronize()
            if self.consumer is not None:
                self.consumer.synchronize()
        self.check()

    def current(self, i: int) -> torch.Tensor:
        """This rank's own loaded window of step ``i`` (the local buffer)."""
        return self.bufs[i % len(self.bufs)].tensor

    # ---- integrity + reporting --------------------------------------------
    def _gather_row(self, vals: List[float], dtype=torch.float64) -> torch.Tensor:
        t = torch.tensor(vals, dtype=dtype, device=self._cdev)
        if self._solo:
            return t.reshape(1, -1).cpu()
        out = torch.empty(self.world * t.numel(), dtype=dtype, device=self._cdev)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out.reshape(self.world, -1).cpu()

    def verify(self, i: Optional[int] = None) -> bool:
        """CRC32C of every slice of the fanned-out window of step ``i``
        (default: the last step; it must still be in the ring) against each
        source rank's host CRC of the file window it loaded.  Collective;
        same verdict on every rank."""
        self.flush()
        i = self.last_step if i is None else i
        mine = file_crc32c(self.path, self.window_offset(i), self.window)
        want = self._gather_row([mine], dtype=torch.int64)[:, 0].tolist()
        if not self.fan:
            ok = crc32c_of(self.bufs[i % len(self.bufs)].tensor) == mine
        else:
            slot = i % self.out_ring
            if self._slot_step[slot] != i:
                raise LookupError(f"step {i} left the ring")
            out = self.outs[slot]
            if self.mode == "allgather":
                W = self.window
                ok = all(crc32c_of(out[r * W:(r + 1) * W]) == want[r] for r in range(self.world))
            else:
                ok = crc32c_of(out) == want[self.src_rank]
        if self._solo:
            return ok
        v = torch.tensor([1 if ok else 0], dtype=torch.int64, device=self._cdev)
        dist.all_reduce(v, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(v.item()) == 1)

    def gather_seconds(self) -> float:
        """Summed device time of this rank's step collectives (the slice
        check included when verify_each)."""
        if self._gather_ev:
            self.side.synchronize()
            s = sum(a.elapsed_time(b) for a, b in self._gather_ev) / 1e3
            self._gather_ev.clear()
            self.gather_s += s
        return self.gather_s

    def crc_seconds(self) -> float:
        """Summed time of this rank's per-step slice checks (verify_each)."""
        if self._crc_ev:
            self.side.synchronize()
            self.crc_s += sum(a.elapsed_time(b) for a, b in self._crc_ev) / 1e3
            self._crc_ev.clear()
        return self.crc_s

    def report(self, wall_s: Optional[float] = None) -> dict:
        """Per-rank load rate, collective time and load/collective overlap
        (collective).  ``overlap`` is the fraction of collective time hidden
        behind loads: (load + gather - wall) / gather, clamped to [0, 1]."""
        wall = self.stats.wall_s if wall_s is None else wall_s
        g = self.gather_seconds()
        row = [self.stats.bytes_loaded / max(self.stats.load_s, 1e-12) / (1 << 30),
               g * 1e3, self.stats.load_s, wall, self.crc_seconds() * 1e3,
               float(self.stats.delivered)]
        allr = self._gather_row(row)
        per_gibps = [round(float(x), 3) for x in allr[:, 0].tolist()]
        per_ms = [round(float(x), 3) for x in allr[:, 1].tolist()]
        overlap = []
        for load_s, gms, w in zip(allr[:, 2].tolist(), allr[:, 1].tolist(), allr[:, 3].tolist()):
            gs = gms / 1e3
            overlap.append(round(min(1.0, max(0.0, (load_s + gs - w) / gs)), 3) if gs > 0 else None)
        return {"load_GiBps_per_rank": per_gibps, "collective_ms_per_rank": per_ms,
                "overlap_per_rank": overlap, "steps": self.stats.steps,
                "bytes_gathered_per_rank": self.stats.bytes_gathered,
                "slice_check_ms_per_rank": [round(float(x), 3) for x in allr[:, 4].tolist()],
                "delivered_steps_per_rank": [int(x) for x in allr[:, 5].tolist()]}

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
