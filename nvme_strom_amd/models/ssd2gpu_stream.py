"""Streaming SSD → HBM loader — the MI355X counterpart of ``nvme_test``.

Reference: utils/nvme_test.c (exec_test_by_strom :383-498, setup_async_tasks
:277-323, callback_dma_wait :208-223).  The reference keeps ``nr_segments``
(6) segments of ``segment_sz`` (32 MiB) in flight, each with its own CUDA
stream and a host callback that blocks in MEMCPY_WAIT.  Here:

* the destination is a resident ``HbmBuffer`` (a window of any size — HBM
  is 288 GB) cut into segments; ``depth`` segments are in flight;
* each segment's MEMCPY_SSD2GPU is issued from the caller thread; the
  engine's own workers move the data (O_DIRECT → pinned staging → SDMA into
  HBM), so no per-segment stream or callback thread is needed;
* WAIT runs on the oldest segment only when the pipeline is full;
* verification is an on-GPU CRC32C per chunk compared with the host CRC of
  the chunk that landed there (no DtoH readback of the data);
* ``vfs_control`` is the reference's ``-f`` mode: pread into pinned memory +
  HtoD (utils/nvme_test.c:501-600), the control the engine must beat.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from .. import api
from ..ops import verify as V
from ..ops.reorder import chunk_scatter, landing_positions
from ..tensor import FileReader, HbmBuffer, _sync, host_buffer


@dataclass
class StreamStats:
    bytes: int = 0
    seconds: float = 0.0
    nr_ram: int = 0
    nr_ssd: int = 0
    nr_submit: int = 0
    nr_blocks: int = 0
    wait_s: float = 0.0
    crc_mismatch: int = 0

    @property
    def gib_per_s(self) -> float:
        return self.bytes / self.seconds / (1 << 30) if self.seconds else 0.0

    @property
    def avg_request_kib(self) -> float:
        return 0.5 * self.nr_blocks / self.nr_submit if self.nr_submit else 0.0


class StreamLoader:
    """Loads file windows into HBM, ``depth`` segments in flight."""

    def __init__(self, path: str, segment_sz: int = 32 << 20, nr_segments: int = 6,
                 chunk_sz: int = 8192, device=None, buf: Optional[HbmBuffer] = None,
                 depth: int = 6):
        self.reader = FileReader(path, chunk_sz=chunk_sz, max_chunks=segment_sz // chunk_sz)
        self.segment_sz = segment_sz
        self.nr_segments = nr_segments
        self.depth = max(1, depth)
        self.chunk_sz = chunk_sz
        self.own_buf = buf is None
        self.buf = buf or HbmBuffer(segment_sz * nr_segments, device)
        self.wbs = [self.reader._wb] + [host_buffer(self.reader._wb.numel())
                                        for _ in range(self.depth - 1)]
        self.stats = StreamStats()
        self.per_seg = segment_sz // chunk_sz

    def run(self, offset: int, nbytes: int, verify: bool = False,
            buf: Optional[HbmBuffer] = None) -> StreamStats:
        """Load file bytes [offset, offset+nbytes) into ``buf`` (default: the
        loader's buffer, wrapping around its segments)."""
        dst = buf or self.buf
        nseg_buf = max(1, dst.nbytes // self.segment_sz)
        st = StreamStats()
        first_chunk = offset // self.chunk_sz
        total_chunks = (nbytes + self.chunk_sz - 1) // self.chunk_sz
        inflight: List[tuple] = []
        t0 = time.perf_counter()
        try:
            for seg, c0 in enumerate(range(0, total_chunks, self.per_seg)):
                if len(inflight) == self.depth:
                    self._retire(inflight.pop(0), st, verify, dst)
                n = min(self.per_seg, total_chunks - c0)
                ids = np.arange(first_chunk + c0, first_chunk + c0 + n, dtype=np.uint32)
                slot = seg % nseg_buf
                res, landed = self.reader.submit(dst, slot * self.segment_sz, ids,
                                                 wb=self.wbs[seg % self.depth])
                inflight.append((res, slot, ids, landed))
            while inflight:
                self._retire(inflight.pop(0), st, verify, dst)
        except BaseException:
            # a failed segment: drain the others before the buffers (and the
            # caller's retry) can be reused, and claim their task records
            for res, *_ in inflight:
                try:
                    self.reader.finish(res)
                except (api.StromError, OSError):
                    pass
            raise
        st.seconds = time.perf_counter() - t0
        st.bytes = nbytes
        self.stats.bytes += st.bytes
        self.stats.seconds += st.seconds
        return st

    def _retire(self, item, st: StreamStats, verify: bool, dst: HbmBuffer) -> None:
        res, slot, ids, landed = item
        w0 = time.perf_counter()
        self.reader.finish(res)
        if res.nr_ram:
            if not np.array_equal(landed, ids):
                # page-cache chunks landed at the tail: restore file order
                lo = slot * self.segment_sz
                region = dst.tensor[lo:lo + len(ids) * self.chunk_sz]
                chunk_scatter(region.clone(), region,
                              landing_positions(ids, landed, res.nr_ssd), self.chunk_sz)
                landed = ids
            # the write-back slot is reused: its HtoD must be complete
            _sync()
        st.wait_s += time.perf_counter() - w0
        st.nr_ram += res.nr_ram
        st.nr_ssd += res.nr_ssd
        st.nr_submit += res.nr_dma_submit
        st.nr_blocks += res.nr_dma_blocks
        if verify:
            st.crc_mismatch += self._verify(dst, slot, landed)

    def _verify(self, dst: HbmBuffer, slot: int, landed) -> int:
        """Per-chunk CRC on the GPU vs host CRC of the chunk each slot holds."""
        lo = slot * self.segment_sz
        seg = dst.tensor[lo:lo + len(landed) * self.chunk_sz]
        dev = V.u32(V.crc32c_chunks(seg, self.chunk_sz))
        bad = 0
        fd = self.reader.fd
        for i, cid in enumerate(landed.tolist()):
            data = os.pread(fd, self.chunk_sz, cid * self.chunk_sz)
            data = data + b"\0" * (self.chunk_sz - len(data))
            if api.crc32c_host(data) != int(dev[i]):
                bad += 1
        return bad

    def close(self) -> None:
        if self.own_buf:
            self.buf.close()
        self.reader.close()


def vfs_control(path: str, offset: int, nbytes: int, buf: torch.Tensor,
                segment_sz: int = 32 << 20, nr_segments: int = 6) -> float:
    """pread → pinned → HtoD ring (nvme_test -f).  Returns seconds."""
    fd = os.open(path, os.O_RDONLY)
    pins = [torch.empty(segment_sz, dtype=torch.uint8, pin_memory=True) for _ in range(nr_segments)]
    evs = [None] * nr_segments
    stream = torch.cuda.Stream()
    t0 = time.perf_counter()
    k = 0
    for off in range(offset, offset + nbytes, segment_sz):
        slot = k % nr_segments
        if evs[slot] is not None:
            evs[slot].synchronize()
        n = min(segment_sz, offset + nbytes - off)
        mv = memoryview(pins[slot].numpy())
        got = os.preadv(fd, [mv[:n]], off)
        dst_off = (k * segment_sz) % buf.numel()
        with torch.cuda.stream(stream):
            buf[dst_off:dst_off + got].copy_(pins[slot][:got], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        evs[slot] = ev
        k += 1
    stream.synchronize()
    dt = time.perf_counter() - t0
    os.close(fd)
    return dt
