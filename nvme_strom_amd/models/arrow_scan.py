"""PG-Strom-style SSD→GPU direct scan of an Apache Arrow IPC file
(BASELINE config 5): file → HBM through the engine → LZ4 decode on the GPU
→ range filter → selected row ids, with no host-side data touch.

Steps
  1. metadata: footer + record-batch headers only (utils/arrow_ipc.py);
  2. load: the whole file (or any byte window) into a resident HBM tensor via
     MEMCPY_SSD2GPU (tensor.load_file);
  3. column: per batch, the data/validity buffers are either zero-copy views
     of the loaded file (uncompressed) or LZ4-frame streams decoded by one
     launch of the GPU decoder into a contiguous column tensor (Arrow's
     BodyCompression: 8-byte uncompressed length prefix, -1 = stored raw);
  4. filter: column_filter per batch (validity ANDed in), bitmap compaction to
     global row ids.
"""
from __future__ import annotations

import os
import struct
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops import decompress as D
from ..ops.colfilter import bitmap_to_indices, column_filter
from ..tensor import load_file
from ..utils.arrow_ipc import ArrowFile, BufferRef, read_metadata

_TORCH = {"i4": torch.int32, "i8": torch.int64, "f4": torch.float32, "f8": torch.float64}


@dataclass
class ScanOut:
    rows: int
    selected: int
    indices: torch.Tensor
    seconds: Dict[str, float]


class ArrowScan:
    def __init__(self, path: str, device=None, chunk_sz: int = 1 << 20):
        self.path = path
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.meta: ArrowFile = read_metadata(path)
        self.chunk_sz = chunk_sz
        self.file: Optional[torch.Tensor] = None
        self._hdr_fd = os.open(path, os.O_RDONLY)
        self.timings: Dict[str, float] = {}

    def load(self) -> torch.Tensor:
        t0 = time.perf_counter()
        self.file = load_file(self.path, self.device, chunk_sz=self.chunk_sz)
        self.timings["load_s"] = time.perf_counter() - t0
        return self.file

    # ----------------------------------------------------------- buffers
    def _buffer_plan(self, ref: BufferRef, codec: Optional[str]) -> Tuple[str, int, int, int, int]:
        """-> (kind, src_off, src_len, out_len, lz4 codec id)"""
        if ref.length == 0:
            return "empty", 0, 0, 0, 0
        if codec is None:
            return "raw", ref.offset, ref.length, ref.length, 0
        if codec != "lz4_frame":
            raise NotImplementedError(f"body compression {codec} (GPU decoder: LZ4 frame)")
        head = os.pread(self._hdr_fd, 32, ref.offset)
        ulen, = struct.unpack_from("<q", head, 0)
        if ulen == -1:
            return "raw", ref.offset + 8, ref.length - 8, ref.length - 8, 0
        info = D.parse_lz4_frame_header(head, 8)
        codec_id = D.LZ4_FRAME_BCS if info.block_checksum else D.LZ4_FRAME
        so = ref.offset + 8 + info.data_offset
        return "lz4", so, ref.length - 8 - info.data_offset, ulen, codec_id

    def _gather(self, refs: List[BufferRef], codecs: List[Optional[str]], sizes: List[int],
                pad_to: int) -> Tuple[torch.Tensor, List[int]]:
        """Materialise buffers back to back (each padded to ``pad_to``)."""
        offs, total = [], 0
        for s in sizes:
            offs.append(total)
            total += (s + pad_to - 1) // pad_to * pad_to
        out = torch.zeros(max(total, 8), dtype=torch.uint8, device=self.device)
        groups: Dict[int, list] = {}
        for ref, codec, o, s in zip(refs, codecs, offs, sizes):
            kind, so, sl, ol, cid = self._buffer_plan(ref, codec)
            if kind == "empty":
                continue
            if kind == "raw":
                n = min(sl, s)
                out[o:o + n].copy_(self.file[so:so + n])
            else:
                groups.setdefault(cid, []).append((so, sl, o, min(ol, s)))
        for cid, items in groups.items():
            st = D.decompress(cid, self.file, out, D.make_descs(items))
            bad = [i for i, (x, it) in enumerate(zip(st, items)) if x != it[3]]
            if bad:
                raise RuntimeError(f"LZ4 decode failed for {len(bad)} buffer(s): {st[bad[:4]]}")
        return out, offs

    def column(self, name: str) -> Tuple[torch.Tensor, Optional[torch.Tensor], List[int]]:
        """(values, validity bytes or None, per-batch row offsets)."""
        if self.file is None:
            self.load()
        ci = self.meta.column_index(name)
        col = self.meta.schema[ci]
        if not col.supported:
            raise NotImplementedError(f"column {name} is not a fixed-width primitive")
        width = col.bit_width // 8
        t0 = time.perf_counter()
        bs = self.meta.batches
        rows = [b.columns[ci].length for b in bs]
        codecs = [b.codec for b in bs]
        # values: back to back, each batch padded to 64 B so views stay aligned
        vals, voffs = self._gather([b.columns[ci].data for b in bs], codecs,
                                   [r * width for r in rows], 64)
        has_nulls = any(b.columns[ci].null_count for b in bs)
        valid = None
        if has_nulls:
            valid, _ = self._gather([b.columns[ci].validity for b in bs], codecs,
                                    [(r + 7) // 8 for r in rows], 64)
        torch.cuda.synchronize() if self.device.type == "cuda" else None
        self.timings["decode_s"] = time.perf_counter() - t0
        self._layout = (voffs, rows, width, col.numpy_dtype)
        return vals, valid, voffs

    def filter(self, name: str, lo, hi) -> ScanOut:
        vals, valid, voffs = self.column(name)
        _, rows, width, dt = self._layout
        t0 = time.perf_counter()
        idx, total, base = [], 0, 0
        voff_valid = 0
        for r, vo in zip(rows, voffs):
            v = vals[vo:vo + r * width].view(_TORCH[dt])
            vb = None
            if valid is not None:
                vb = valid[voff_valid:voff_valid + ((r + 7) // 8 + 63) // 64 * 64]
                voff_valid += ((r + 7) // 8 + 63) // 64 * 64
            bm, cnt = column_filter(v, lo, hi, vb)
            if cnt:
                idx.append(bitmap_to_indices(bm, r, cnt).to(torch.int64) + base)
            total += cnt
            base += r
        out = torch.cat(idx) if idx else torch.zeros(0, dtype=torch.int64, device=self.device)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        self.timings["filter_s"] = time.perf_counter() - t0
        return ScanOut(base, total, out, dict(self.timings))

    def close(self) -> None:
        if self._hdr_fd >= 0:
            os.close(self._hdr_fd)
            self._hdr_fd = -1
