"""PG-Strom-style SSD→GPU direct scan of an Apache Arrow IPC file
(BASELINE config 5): only the scanned column's buffers travel storage → HBM
through the engine, are LZ4-decoded and filtered on the GPU, and the
selected row ids are appended on the device — one host sync per scan.

Pipeline (a ring of ``nslots`` HBM slots, groups of record batches):

    host:   plan groups from the footer / batch headers (utils/arrow_ipc.py):
            per batch the column's data (+ validity when it has nulls)
            buffer ranges -> the file chunks that cover them
    group g:  MEMCPY_SSD2GPU(chunk ids of g) -> slot g % nslots      (engine)
              WAIT(g) ; then on the slot's stream, no host sync:
                decode  one launch over every compressed buffer of g
                        (Arrow BodyCompression LZ4_FRAME: the length prefix and
                        frame header are parsed on the device);
                        status vs expected sizes -> device error counter
                filter  one launch over every batch of g (validity ANDed in,
                        each batch on fresh bitmap words), count on device
                emit    global row ids appended at a device-side cursor, on one
                        emit stream in group order (decode/filter of several
                        groups run concurrently on their slots' streams)
              event(g) ; the slot is refilled only after event(g)
    while group g computes, group g+1 is already being read.

Unreferenced columns are never read; files larger than HBM stream through
the ring.  The reference has no columnar path (new MI355X
work); its chunk-list I/O (MEMCPY_SSD2GPU with arbitrary chunk ids,
kmod/nvme_strom.c:1488-1604) is what fetches the scattered buffers.
"""
from __future__ import annotations

import os
import struct
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import api
from ..ops import decompress as D
from ..ops.colfilter import BATCH_FIELDS, bitmap_to_rows, bitmap_to_rows_str
from ..ops.colpred import (QUAL_BATCH_FIELDS, Compiled, Pred, clauses, compile_pred, evaluate,
                           qual_batched)
from ..ops.reorder import chunk_scatter, landing_positions
from ..tensor import FileReader, HbmBuffer, host_buffer
from ..utils.arrow_ipc import (ArrowFile, Column, _Src, decode_values, dictionary_values,
                               read_buffer, read_metadata, validity_bits)

# projection output dtypes by storage (date/time/timestamp/duration: their
# integer ticks; dictionary-encoded: the indices)
_TORCH = {"i1": torch.int8, "u1": torch.uint8, "i2": torch.int16, "u2": torch.uint16,
          "i4": torch.int32, "u4": torch.uint32, "i8": torch.int64, "u8": torch.uint64,
          "f4": torch.float32, "f8": torch.float64}


@dataclass
class ScanOut:
    rows: int
    selected: int
    indices: torch.Tensor
    seconds: Dict[str, float]
    bytes_read: int = 0           # file bytes moved storage -> HBM
    column_bytes: int = 0         # decoded bytes of the scanned columns
    groups: int = 0
    values: Optional[torch.Tensor] = None   # projected column, one value per selected row
    valid: Optional[torch.Tensor] = None    # its validity (uint8 0/1) when it has nulls
    column: Optional[Column] = None         # the projected column's type (units, tz, ...)
    dictionary: object = None               # its decoded dictionary when dictionary-encoded
    offsets: Optional[torch.Tensor] = None  # utf8/binary projection: int64[selected + 1]
                                            # into ``values`` (the characters, uint8)


@dataclass
class _Buf:
    off: int          # file offset of the stored buffer
    length: int       # stored bytes (prefix + frame when compressed)
    need: int         # bytes the scan reads from the decoded buffer
    cap: int          # decode capacity (need rounded up to 64)
    compressed: bool


@dataclass
class _Batch:
    rows: int
    row_base: int
    # per scanned column: (data, validity, extra) — data: values / bool bits /
    # dictionary indices / utf8-binary offsets; extra: the characters
    cols: List[Tuple[_Buf, Optional[_Buf], Optional[_Buf]]]


class _PlanArr:
    """The plan as arrays (no per-batch Python objects: a cold qualifier-list
    plan over thousands of record batches was ~0.1 s of Python): per batch
    ``rows`` / ``row_base``, per (batch, column, buffer) with buffer 0 data,
    1 validity, 2 characters: file ``off``, stored ``length``, decoded
    ``need``, decode ``cap`` and ``present``; ``comp`` per batch.  Indexing
    gives the _Batch view of one batch; slicing a range of batches."""

    def __init__(self, rows, row_base, off, length, need, cap, present, comp):
        self.rows, self.row_base = rows, row_base
        self.off, self.length, self.need, self.cap = off, length, need, cap
        self.present, self.comp = present, comp

    def __len__(self) -> int:
        return len(self.rows)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return _PlanArr(*(a[i] for a in (self.rows, self.row_base, self.off, self.length,
                                             self.need, self.cap, self.present, self.comp)))
        cols = []
        for k in range(self.off.shape[1]):
            cols.append(tuple(_Buf(int(self.off[i, k, j]), int(self.length[i, k, j]),
                                   int(self.need[i, k, j]), int(self.cap[i, k, j]),
                                   bool(self.comp[i])) if self.present[i, k, j] else None
                              for j in range(3)))
        return _Batch(int(self.rows[i]), int(self.row_base[i]), cols)

    def __iter__(self):
        return (self[i] for i in range(len(self)))


@dataclass
class _Group:
    b0: int                               # batches [b0, b1) of the scanned range
    b1: int
    ids: np.ndarray                       # sorted file chunk ids
    dec_bytes: int = 0
    words: int = 0
    # slot-relative launch tables, built once per plan (_prepare): decoder
    # descriptors, and per batch and column the data/validity pointers as
    # (kind, offset) with kind 0 none, 1 slot region, 2 decode buffer
    descs: Optional[np.ndarray] = None
    need: Optional[np.ndarray] = None
    descs_lanes: Optional[np.ndarray] = None   # literal-heavy LZ4 buffers (lane decoder)
    need_lanes: Optional[np.ndarray] = None
    ptr_kind: Optional[np.ndarray] = None   # (n, ncols, 3)
    ptr_rel: Optional[np.ndarray] = None    # (n, ncols, 3)
    aux_len: Optional[np.ndarray] = None    # (n, ncols) decoded character bytes
    table: Optional[np.ndarray] = None      # (n, QUAL_BATCH_FIELDS), pointer columns 0
    column_bytes: int = 0
    has_valid: Optional[np.ndarray] = None  # (ncols,) some batch has a validity buffer
    # extent reads (ArrowScan.EXTENTS): the group's buffers as strom_file_extent
    # records in file order with their slot offsets, the slot span they take
    # and the bytes the reads cover (buffers + holes read through + padding)
    ext: Optional[np.ndarray] = None
    span: int = 0
    read_bytes: int = 0
    gap_bytes: int = 0


@dataclass
class _Slot:
    off: int                               # byte offset of the slot in the ring buffer
    cap: int                               # slot bytes
    dec: torch.Tensor
    bitmap: torch.Tensor
    bm2: Optional[torch.Tensor] = None     # OR-clause scratch bitmap
    event: Optional[torch.cuda.Event] = None
    stream: Optional[torch.cuda.Stream] = None
    count: Optional[torch.Tensor] = None   # selected rows of the slot's group
    junk: Optional[torch.Tensor] = None    # counts of non-final qualifiers
    err: Optional[torch.Tensor] = None     # failed decodes of the slot's group
    scratch: Optional[torch.Tensor] = None # chunk-order restore (page-cache hits)
    pending: object = None                # (CopyResult, landed ids, group)
    keep: List[torch.Tensor] = field(default_factory=list)
    pin: Optional[torch.Tensor] = None     # pinned arena for the group's tables
    pin_off: int = 0


def _up64(n: int) -> int:
    return (n + 63) // 64 * 64


def _up64_np(n: np.ndarray) -> np.ndarray:
    return (n + 63) // 64 * 64


def _stored_sizes(path: str, off: np.ndarray, ln: np.ndarray, comp: np.ndarray) -> np.ndarray:
    """Decoded bytes of variable-size buffers (utf8/binary characters):
    the stored length when raw, else the Arrow BodyCompression prefix
    (i64 uncompressed length, -1 = stored raw after it), read with a few
    preads in flight — the plan needs the decode capacity before any data
    is read into HBM."""
    out = np.asarray(ln, np.int64).copy()
    comp = np.asarray(comp, bool)
    out[comp & (out < 8)] = 0
    idx = np.flatnonzero(comp & (np.asarray(ln) >= 8))
    if len(idx):
        from concurrent.futures import ThreadPoolExecutor
        fd = os.open(path, os.O_RDONLY)
        try:
            with ThreadPoolExecutor(16) as ex:
                vals = np.array(list(ex.map(
                    lambda o: struct.unpack("<q", os.pread(fd, 8, o))[0],
                    np.asarray(off)[idx].tolist())), dtype=np.int64)
        finally:
            os.close(fd)
        raw = vals == -1
        bad = ~raw & ((vals < 0) | (vals >= (1 << 31)))
        if bad.any():
            k = int(idx[np.flatnonzero(bad)[0]])
            raise ValueError(f"record batch {k}: buffer length prefix {int(vals[bad][0])}")
        out[idx] = np.where(raw, out[idx] - 8, vals)
    return out


class ArrowScan:
    # the decoder runs one stream per compressed buffer at a roughly fixed
    # per-stream rate (profiles/r2/dec): a launch needs thousands of streams
    # to fill the GPU, so compressed groups grow to hold that many buffers
    TARGET_STREAMS = 8192
    # streams per group: one round of the block-parallel decoder's resident
    # workgroups (its 512-thread build: 3 per CU, 768 config-5 frames at
    # 115 GB/s), so a group's decode takes one stream's latency and the last
    # group's decode — the part no read overlaps — stays short.  0: cut a
    # compressed column into nslots groups instead.  (Same-box A/B of 2 / 4
    # per CU and 0 on config 5 was inside the storage noise:
    # profiles/r3/arrow_group_policy_ab/.)
    ROUND_STREAMS_PER_CU = int(os.environ.get("STROM_ARROW_ROUND_PER_CU", "3"))
    # ZSTD groups: 1 / ZSTD_ROUND_DIV of the zstd decoder's resident round
    # (lane-parallel decoder: 2, four groups for config 5's val — its
    # decode latency is per block, so a group's decode overlaps the next
    # groups' reads; 4+ groups lose to the reads' interleaving)
    ZSTD_ROUND_DIV = int(os.environ.get("STROM_ARROW_ZSTD_DIV", "2"))
    # the zstd decoder per group launch: 2 lane-parallel (default: the
    # blocks' entropy stages on the lanes of a wave, so a group's decode
    # takes about one block's latency, not one stream's), None the wave /
    # frame-parallel choice by stream count, 0 one wave per stream, 1
    # frame-parallel
    ZSTD_MODE = (int(os.environ["STROM_ARROW_ZSTD_MODE"])
                 if os.environ.get("STROM_ARROW_ZSTD_MODE") else 2)
    # reads: the group's buffers as exact extents (MEMCPY_SSD2GPU_EXTENTS,
    # VERDICT r5 #4) — a column's buffers in large requests, holes up to
    # EXTENT_GAP read through — instead of the fixed-size chunk ids covering
    # them (whole chunks: read amplification, small scattered requests).
    # STROM_ARROW_EXTENTS=0: chunk ids (A/B)
    EXTENTS = os.environ.get("STROM_ARROW_EXTENTS", "1") != "0"
    EXTENT_GAP = int(os.environ.get("STROM_ARROW_EXTENT_GAP", str(64 << 10)))

    def __init__(self, path: str, device=None, chunk_sz: Optional[int] = None,
                 slot_bytes: int = 256 << 20, nslots: Optional[int] = None,
                 max_slot_bytes: int = 4 << 30):
        """``chunk_sz`` / ``nslots`` default by the file's codec: LZ4 64 KiB
        chunks, 3 slots; ZSTD 16 KiB chunks (a buffer is read as whole
        chunks: 600 -> 500 MB read for config 5's ``val``) and 4 slots, so
        the reads of every one of its groups are in flight behind the first
        (profiles/r5/zstd_arrow/group_ab/)."""
        self.path = path
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.meta: ArrowFile = read_metadata(path)
        zstd = set(self.meta.codecs) - {None} == {"zstd"}
        self.chunk_sz = chunk_sz if chunk_sz else ((16 << 10) if zstd else (64 << 10))
        self.slot_bytes = slot_bytes
        self.max_slot_bytes = max(slot_bytes, max_slot_bytes)
        self.nslots = max(2, nslots if nslots else (4 if zstd else 3))
        self.reader: Optional[FileReader] = None
        self._slots: List[_Slot] = []
        self._wbs: List[Optional[torch.Tensor]] = []
        # (column tuple, batch range) -> (dtypes, rows, groups)
        self._plans: Dict[tuple, tuple] = {}
        self._bplans: Dict[tuple, tuple] = {}   # column tuple -> _plan()
        self._dicts: Dict[str, tuple] = {}      # decoded dictionaries
        self._compiled: Dict[tuple, Compiled] = {}

    # ------------------------------------------------------------- plan
    def _plan(self, names: Sequence[str]) -> tuple:
        """(per batch _Batch with each column's (data, validity, extra)
        buffers, the Column metas, total rows).  data: the values / bool
        bits / dictionary indices / utf8-binary offsets; extra: the
        characters of a utf8/binary column."""
        cis, cols = [], []
        for name in names:
            ci = self.meta.column_index(name)
            col = self.meta.schema[ci]
            if not col.supported:
                raise NotImplementedError(f"column {name}: {col.kind} columns are not scanned "
                                          "on the GPU")
            cis.append(ci)
            cols.append(col)
        m = self.meta
        used = set(m.codecs) - {None}
        if not used <= {"lz4_frame", "zstd"} or len(used) > 1:
            raise NotImplementedError(f"body compression {sorted(used)} (GPU decoders: one of "
                                      "LZ4 frame, ZSTD per file)")
        # lz4par.hip / zstd.hip (Arrow IPC buffer codecs: length prefix + frame)
        self._codec = D.ARROW_ZSTD if used == {"zstd"} else D.ARROW_LZ4
        comp = np.array([c is not None for c in m.codecs], dtype=bool)
        rows = m.columns[cis[0]].length if m.nbatches else np.zeros(0, np.int64)
        base = np.concatenate([[0], np.cumsum(rows)]).astype(np.int64)
        nb, nc = len(rows), len(cols)
        off = np.zeros((nb, nc, 3), np.int64)
        length = np.zeros((nb, nc, 3), np.int64)
        need = np.zeros((nb, nc, 3), np.int64)
        present = np.zeros((nb, nc, 3), bool)
        for k, (ci, col) in enumerate(zip(cis, cols)):
            a = m.columns[ci]
            n = a.length
            st = col.storage
            if st == "b1":
                dneed = (n + 7) // 8
            elif st == "d16":
                dneed = n * 16
            elif col.kind in ("utf8", "binary") and col.dictionary is None:
                dneed = np.where(n > 0, (n + 1) * (8 if col.large else 4), 0)
            else:
                dneed = n * np.dtype(st).itemsize
            strings = a.x_off is not None and col.dictionary is None
            xneed = _stored_sizes(self.path, a.x_off, a.x_len, comp) if strings else None
            for what, o, ln, nd in (("data", a.d_off, a.d_len, dneed),
                                    ("characters", a.x_off, a.x_len, xneed)):
                if nd is None:
                    continue
                # a raw buffer shorter than its rows, or an empty one (compressed
                # or not) for a non-empty batch, would send the kernels past
                # the bytes the plan reserves for it
                short = (~comp & (ln < nd)) | ((ln == 0) & (nd > 0))
                if short.any():
                    b = int(np.flatnonzero(short)[0])
                    raise ValueError(f"column {col.name}, record batch {b}: {what} buffer of "
                                     f"{int(ln[b])} bytes for {int(nd[b])}")
            off[:, k, 0], length[:, k, 0], need[:, k, 0] = a.d_off, a.d_len, dneed
            present[:, k, 0] = True
            off[:, k, 1], length[:, k, 1], need[:, k, 1] = a.v_off, a.v_len, (n + 7) // 8
            present[:, k, 1] = (a.null_count != 0) & (a.v_len != 0)
            if strings:
                off[:, k, 2], length[:, k, 2], need[:, k, 2] = a.x_off, a.x_len, xneed
                present[:, k, 2] = True
        # decode capacities: data / characters rounded up to 64, validity
        # + 64 (the filters read it as whole 64-bit words)
        cap = _up64_np(need)
        cap[:, :, 1] += 64
        cap[:, :, 2] += 64
        plan = _PlanArr(rows.astype(np.int64), base[:-1], off, length, need, cap, present, comp)
        return plan, cols, int(base[-1])

    def _round_streams(self) -> int:
        cus = 256
        if self.device.type == "cuda":
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        if getattr(self, "_codec", None) == D.ARROW_ZSTD:
            # zstd.hip: one wavefront per stream, residency bound by its LDS.
            # A group's decode takes about one stream's latency whatever its
            # size (the entropy stage is serial per stream), so groups stay a
            # whole round: smaller ones queue on the HBM slot ring one
            # latency each (A/B, profiles/r3/zstd/arrow_group_div_ab.json:
            # val 11.0-12.8 GB/s at a round, 5.8 at a quarter, 4.2 at an eighth)
            from .. import _native as N
            if self.ZSTD_MODE == 2:
                # lane-parallel: a group of about one resident round of its
                # entropy waves' blocks (config-5 buffers: 4 blocks each)
                info = np.zeros(8, np.uint32)
                N.lib().strom_zstd_lp_info(info.ctypes.data)
                rnd = cus * int(info[2]) * int(info[1]) // 4
            elif self.ZSTD_MODE == 1:             # frame-parallel: its own round
                rnd = cus * max(1, int(N.lib().strom_zstd_fp_per_cu()))
            else:
                rnd = cus * max(1, (160 << 10) // int(N.lib().strom_zstd_lds_bytes()))
            return max(1, rnd // self.ZSTD_ROUND_DIV)
        return self.ROUND_STREAMS_PER_CU * cus

    def _groups(self, pl: _PlanArr) -> List[_Group]:
        slot = self.slot_bytes
        nb = len(pl)
        # really compressed buffers (a stored-raw one is as long as its data)
        # (zstd: every compressed buffer takes the entropy stage's latency,
        # however little it compressed — only stored ones are skipped)
        lim = 1.0 if getattr(self, "_codec", None) == D.ARROW_ZSTD else 0.9
        d_len, d_need = pl.length[:, :, 0], pl.need[:, :, 0]
        real = pl.comp[:, None] & (d_len > 0) & (d_len < lim * d_need)     # (nb, ncols)
        ncomp = int(real.sum())
        if ncomp:
            # few streams per launch are fine for the block-parallel decoder
            # (lz4par.hip: a workgroup per stream), so a column of many
            # buffers is cut into nslots groups: the decode of group g then
            # overlaps the reads of groups g+1.. (with the round-2 lane
            # decoder every launch took one serial stream's time and the
            # split measured slower, profiles/r3/arrow_split3.json)
            stored = pl.present & (pl.length > 0)
            total = float((pl.length * stored * real[:, :, None]).sum())
            avg = total / ncomp
            want = avg * self.TARGET_STREAMS
            # groups of at most one resident round of streams: the decode of
            # a group takes one stream's latency, and the last group's
            # decode (the part no read overlaps) is as short as it gets
            rnd = self._round_streams()
            if rnd and ncomp > rnd:
                slot = int(min(self.max_slot_bytes, want, total / -(-ncomp // rnd) * 1.02))
            else:
                if not rnd and ncomp >= self.nslots * 256:
                    want = min(want, total / self.nslots)     # one group per slot
                slot = int(min(self.max_slot_bytes, max(slot, want)))
        limit = max(1, slot // self.chunk_sz)
        # (batch, chunk) pairs of every stored buffer, in file order: record
        # batch bodies follow each other, so chunk ids never decrease from one
        # batch to the next, and the distinct chunks of batches [a, b] are
        # the "new" pairs among theirs (prefix sums: no per-batch sets)
        c = self.chunk_sz
        st = pl.present & (pl.length > 0)
        bi, ki, ji = np.nonzero(st)
        lo = pl.off[bi, ki, ji] // c
        hi = (pl.off[bi, ki, ji] + pl.length[bi, ki, ji] + c - 1) // c
        cnt = hi - lo
        tot = int(cnt.sum())
        pb = np.repeat(bi, cnt)
        start = np.repeat(np.cumsum(cnt) - cnt, cnt)
        ch = np.repeat(lo, cnt) + (np.arange(tot) - start)
        order = np.lexsort((ch, pb))
        pb, ch = pb[order], ch[order]
        if tot:
            keep = np.ones(tot, bool)
            keep[1:] = (pb[1:] != pb[:-1]) | (ch[1:] != ch[:-1])
            pb, ch = pb[keep], ch[keep]
        new = np.ones(len(ch), bool)
        if len(ch):
            new[1:] = ch[1:] != ch[:-1]
        cum = np.concatenate([[0], np.cumsum(new)])
        first = np.searchsorted(pb, np.arange(nb), "left")
        last = np.searchsorted(pb, np.arange(nb), "right")
        bounds = []
        a = 0
        firstl, lastl, cuml = first.tolist(), last.tolist(), cum.tolist()
        for b in range(nb):
            s0, e1 = firstl[a], lastl[b]
            # distinct chunks of batches [a, b]: the first pair counts too
            d = (cuml[e1] - cuml[s0 + 1] + 1) if e1 > s0 else 0
            if b > a and d > limit:
                bounds.append((a, b))
                a = b
        if nb:
            bounds.append((a, nb))
        groups = []
        for a, b in bounds:
            ids = np.unique(ch[first[a]:last[b - 1]]).astype(np.int64)
            g = _Group(a, b, ids)
            sub = pl[a:b]
            g.dec_bytes = int((sub.cap * (sub.present & sub.comp[:, None, None])).sum())
            g.words = int(((sub.rows + 63) // 64).sum())
            self._prepare(g, sub)
            groups.append(g)
        return groups

    def _prepare(self, g: _Group, pl: _PlanArr) -> None:
        c = self.chunk_sz
        n, ncols = pl.off.shape[0], pl.off.shape[1]
        pres = pl.present
        comp3 = np.broadcast_to(pl.comp[:, None, None], pres.shape)
        empty = pres & (pl.length == 0)               # empty batch: nothing is read
        dec = pres & ~empty & comp3
        raw = pres & ~empty & ~comp3
        kind = np.zeros((n, ncols, 3), np.int8)
        kind[empty | dec] = 2
        kind[raw] = 1
        rel = np.zeros((n, ncols, 3), np.int64)
        # decode buffer offsets in (batch, column, buffer) order
        capd = np.where(dec, pl.cap, 0).reshape(-1)
        dstart = (np.cumsum(capd) - capd).reshape(n, ncols, 3)
        rel[dec] = dstart[dec]

        if self.EXTENTS:
            # the group's buffers as extents in file order, laid out by the
            # engine's planner (plan only: the slot offsets and span)
            stm = pres & (pl.length > 0)
            eo, el = pl.off[stm].astype(np.int64), pl.length[stm].astype(np.int64)
            order = np.argsort(eo, kind="stable")
            eo, el = eo[order], el[order]
            uo, first = np.unique(eo, return_index=True)
            ul = np.maximum.reduceat(el, first) if len(uo) else el[:0]
            g.ext = api.extents_array(uo, ul)
            r = api.memcpy_ssd2gpu_extents(0, 0, self._plan_fd(), g.ext, gap_max=self.EXTENT_GAP,
                                           plan_only=True)
            g.span = int(-(-r.dst_bytes // 4096) * 4096)
            g.read_bytes, g.gap_bytes = int(r.bytes_read), int(r.gap_bytes)

            def slot_off(off):
                off = np.asarray(off, dtype=np.int64)
                return g.ext["dst_off"][np.searchsorted(uo, off)].astype(np.int64)
        else:
            # file offsets -> offsets in the slot (chunks land in id order)
            def slot_off(off):
                off = np.asarray(off, dtype=np.int64)
                return np.searchsorted(g.ids, off // c) * c + off % c
            g.span = len(g.ids) * c
            g.read_bytes = g.span
        rel[raw] = slot_off(pl.off[raw])
        g.descs = g.descs_lanes = None
        # LZ4 buffers that barely compressed (>= 0.9 of their data: long
        # literal runs, e.g. a utf8 column's characters) go to the
        # lane-group decoder, which copies literals wide and parses their
        # few tokens serially; the block-parallel one is for the rest
        # (lz4par_bench chars: lanes 174 / par 109 GB/s at 2,048 streams;
        # val: lanes 28 / par 109)
        lit = dec & (pl.length >= 0.9 * pl.need) if self._codec == D.ARROW_LZ4 else \
            np.zeros_like(dec)
        for m, attr in ((dec & ~lit, "descs"), (lit, "descs_lanes")):
            if not m.any():
                continue
            # largest decodes first: a stream's decode time grows with its
            # size, and the decoders hand streams to workgroups in descriptor
            # order (zstd.hip's persistent grid takes stream w, w + grid, ...),
            # so the small validity buffers fill in behind the data buffers
            # instead of taking a resident round of their own
            dl = pl.cap[m]
            order = np.argsort(-dl, kind="stable")
            setattr(g, attr, D.make_descs_arrays(slot_off(pl.off[m])[order], pl.length[m][order],
                                                 dstart[m][order], dl[order]))
            setattr(g, "need" if attr == "descs" else "need_lanes",
                    pl.need[m].astype(np.int32)[order])
        g.ptr_kind, g.ptr_rel = kind, rel
        g.aux_len = np.where(pres[:, :, 2], pl.need[:, :, 2], 0)
        words = (pl.rows + 63) // 64
        table = np.zeros((n, QUAL_BATCH_FIELDS), dtype=np.int64)
        table[:, 2] = pl.rows
        table[:, 3] = np.concatenate([[0], np.cumsum(words)[:-1]]) if n else 0
        table[:, 4] = pl.row_base
        g.table = table
        # decoded bytes the scan reads: values / indices / offsets + characters
        g.column_bytes = int(pl.need[:, :, 0].sum() + (pl.need[:, :, 2] * pres[:, :, 2]).sum())
        g.has_valid = pres[:, :, 1].any(axis=0)

    # --------------------------------------------------------- pipeline
    # HBM for the slot ring beyond nslots (a slot per group up to this):
    # with a slot of its own a group's read never waits for an earlier
    # group's decode to free one (r5 timeline: date_ts group 4 was submitted
    # 12 ms late, behind group 0's decode, and held groups 2-3's launches)
    MAX_RING_BYTES = 8 << 30
    MAX_SLOTS = 16
    # HBM for everything a slot holds: its compressed ring share, its decode
    # buffer and (ZSTD lane-parallel) the entry pool the library keeps for
    # its stream (only the ring was counted)
    MAX_SLOT_HBM = 48 << 30

    def _lp_pool_bytes(self, dec: int) -> int:
        """The LP decoder's entry pool for a decode of ``dec`` bytes
        (zstd.hip strom_decompress_zstd_lp: STROM_ZSTD_LP_ENT x dst + block
        and stream tables), 0 for other decoders."""
        if getattr(self, "_codec", None) != D.ARROW_ZSTD or self.ZSTD_MODE != 2:
            return 0
        f = float(os.environ.get("STROM_ZSTD_LP_ENT") or 0) or 3.0
        return int(f * dec) + (1 << 20) + dec // 32768 * 64

    def _slot_count(self, groups: List[_Group], nbytes: int, dec: int = 0) -> int:
        """Slots of the HBM ring: one per group while they fit MAX_RING_BYTES
        / MAX_SLOTS and, with their decode buffers and LP pools, MAX_SLOT_HBM;
        never fewer than nslots (or than the groups).  ZSTD lane-parallel
        slots are also capped by the pools the library keeps per stream
        (strom_zstd_scratch_keep): one more slot would evict another slot's
        pool every decode — a hipFree that waits for the device, and a
        multi-GB hipMalloc.  The read-ahead stays nslots - 1 groups."""
        n = len(groups)
        per_slot = nbytes + dec + self._lp_pool_bytes(dec)
        fit = max(1, min(self.MAX_SLOTS, self.MAX_RING_BYTES // max(nbytes, 1),
                         self.MAX_SLOT_HBM // max(per_slot, 1)))
        want = max(1, min(n, max(self.nslots, fit)))
        if self._lp_pool_bytes(dec):
            from .. import _native as N
            want = min(want, max(1, int(N.lib().strom_zstd_scratch_keep())))
        return want

    def _plan_fd(self) -> int:
        """A descriptor of the file for the extent planner (file size)."""
        if getattr(self, "_pfd", None) is None:
            self._pfd = os.open(self.path, os.O_RDONLY)
        return self._pfd

    def _ensure_slots(self, groups: List[_Group]) -> None:
        nbytes = max(max(g.span for g in groups), self.chunk_sz)
        nbytes = -(-nbytes // self.chunk_sz) * self.chunk_sz
        dec = max(max(g.dec_bytes for g in groups), 64)
        words = max(max(g.words for g in groups), 1)
        want_slots = self._slot_count(groups, nbytes, dec)
        if self._slots and len(self._slots) >= want_slots and (
                self._slots[0].cap >= nbytes and
                            self._slots[0].dec.numel() >= dec and
                            self._slots[0].bitmap.numel() >= words):
            return
        self._free_slots()
        # one registered HBM ring for every slot: one MAP (dma-buf export +
        # BAR mapping) per scan object instead of one per slot (cold cost);
        # no more slots than groups
        nsl = want_slots
        self._hbm = HbmBuffer(nbytes * nsl, self.device)
        for k in range(nsl):
            sl = _Slot(k * nbytes, nbytes,
                       torch.empty(dec, dtype=torch.uint8, device=self.device),
                       torch.empty(words, dtype=torch.int64, device=self.device),
                       torch.empty(words, dtype=torch.int64, device=self.device))
            sl.stream = torch.cuda.Stream(device=self.device)
            sl.count = torch.zeros(1, dtype=torch.int64, device=self.device)
            sl.junk = torch.zeros(1, dtype=torch.int64, device=self.device)
            sl.err = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._slots.append(sl)
        if self.reader is None:
            self.reader = FileReader(self.path, chunk_sz=self.chunk_sz,
                                     max_chunks=nbytes // self.chunk_sz)
        # pinned write-back buffers only once the BAR path is refused (a
        # cold-scan cost otherwise: GiBs of pinned host memory per scan)
        self._wbs = [None] * len(self._slots)
        self._wb_bytes = nbytes

    def _submit(self, k: int, g: _Group) -> None:
        s = self._slots[k % len(self._slots)]
        if s.event is not None:
            s.event.synchronize()            # the slot's previous group is consumed
            s.event = None
        s.keep = []
        # the slot's own write-back buffer, sized for this scan's groups and
        # pinned only if page-cache chunks have to go through host memory
        # (a group may outgrow the reader's own buffer, and slots in flight
        # must not share one)
        i = k % len(self._wbs)

        def wb():
            if self._wbs[i] is None:
                self._wbs[i] = host_buffer(self._wb_bytes)
            return self._wbs[i]
        if self.EXTENTS:
            res = api.memcpy_ssd2gpu_extents(self._hbm.handle, s.off, self.reader.fd, g.ext,
                                             gap_max=self.EXTENT_GAP, sess=self.reader.sess)
            s.pending = (res, None, g)
            return
        res, landed = self.reader.submit(self._hbm, s.off, g.ids.astype(np.uint32), wb=wb)
        s.pending = (res, landed, g)

    @staticmethod
    def _pointers(g: _Group, col: int, base: int, dec_base: int) -> np.ndarray:
        """The group's strom_qual_batch table for one column: values,
        validity and character pointers resolved against this slot."""
        t = g.table.copy()
        kind, rel = g.ptr_kind[:, col, :], g.ptr_rel[:, col, :]
        ptrs = np.where(kind == 1, base + rel, np.where(kind == 2, dec_base + rel, 0))
        t[:, 0], t[:, 1], t[:, 5] = ptrs[:, 0], ptrs[:, 1], ptrs[:, 2]
        t[:, 6] = g.aux_len[:, col]
        return t

    def _upload(self, s: "_Slot", arr: np.ndarray) -> torch.Tensor:
        """``arr`` as a device tensor, copied on the current stream through
        the slot's pinned arena.  A pinned allocation per group (pin_memory())
        could synchronize the device: the host then waited for group k's
        decode before launching group k+1's (r5 Arrow ZSTD timeline: 12.7 ms
        between group 1 landing and its launch).  The arena is reused once
        the slot's previous group is consumed (_submit waits for it)."""
        a = np.ascontiguousarray(arr)
        raw = a.reshape(-1).view(np.uint8)
        n = raw.nbytes
        o = (s.pin_off + 255) & ~255
        if s.pin is None or o + n > s.pin.numel():
            if s.pin is not None:
                s.keep.append(s.pin)          # earlier copies of this group read it
            s.pin = torch.empty(max(4 << 20, 2 * (n + 256)), dtype=torch.uint8,
                                pin_memory=self.device.type == "cuda")
            o = 0
        s.pin_off = o + n
        host = s.pin[o:o + n]
        host.numpy()[:] = raw
        d = torch.empty(n, dtype=torch.uint8, device=self.device)
        d.copy_(host, non_blocking=True)
        return d.view(torch.from_numpy(a[:0].reshape(-1)).dtype).reshape(a.shape)

    def _compute(self, k: int, spec, proj, state) -> None:
        s = self._slots[k % len(self._slots)]
        res, landed, g = s.pending
        s.pending = None
        s.pin_off = 0
        t0 = time.perf_counter()
        self.reader.finish(res)
        t1 = time.perf_counter()
        state["wait_s"] += t1 - t0
        state["marks"].append((k, "landed", t1))
        region = self._hbm.tensor[s.off:s.off + g.span]
        nr_ram = getattr(res, "nr_ram", 0)            # extent reads: all from storage
        # write-back copies of page-cache chunks (FileReader.submit without a
        # BAR) were queued on the current stream; only then wait for it (a
        # wait on the default stream also waits for whatever blocking
        # streams hold)
        cs = s.stream
        if nr_ram:
            cs.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(cs):
            if nr_ram and not np.array_equal(landed, g.ids.astype(np.uint32)):
                # page-cache chunks landed at the tail: restore chunk order
                if s.scratch is None:
                    s.scratch = torch.empty(s.cap, dtype=torch.uint8, device=self.device)
                tmp = s.scratch[:region.numel()]
                tmp.copy_(region)
                chunk_scatter(tmp, region, landing_positions(g.ids.astype(np.uint32), landed,
                                                             res.nr_ssd), self.chunk_sz)
            base = region.data_ptr()
            dec_base = s.dec.data_ptr()
            descs = g.descs if g.descs is not None else g.descs_lanes
            for dsc, need, lanes in ((g.descs, g.need, False), (g.descs_lanes, g.need_lanes, True)):
                if dsc is None:
                    continue
                # every compressed buffer of every scanned column: one launch
                # (two when some are literal-heavy LZ4)
                d_desc = self._upload(s, dsc.view(np.uint8))
                d_need = self._upload(s, need)
                status = torch.empty(len(dsc), dtype=torch.int32, device=self.device)
                D.decompress_async(self._codec, region, s.dec, d_desc, status, stream=cs,
                                   lanes=lanes, zstd_mode=self.ZSTD_MODE)
                # status = decoded bytes; short or failed -> error count
                s.err += ((status < d_need) | (status < 0)).sum()
                s.keep += [d_desc, d_need, status]
                state["marks"].append((k, "decode_queued", time.perf_counter()))
            # one batch table per referenced column, uploaded once per group
            tabs: Dict[int, torch.Tensor] = {}

            def table(col: int) -> torch.Tensor:
                if col not in tabs:
                    t = self._pointers(g, col, base, dec_base)
                    tabs[col] = self._upload(s, t)
                    s.keep.append(tabs[col])
                return tabs[col]
            # the CNF qualifier list: clause 0 writes the bitmap (its
            # predicates ORed in place), a later single-predicate clause ANDs
            # into it, a later OR-clause collects in the scratch bitmap and
            # its last predicate ORs that in and ANDs into the bitmap; the
            # last launch's count is the selection's
            for ci, clause in enumerate(spec):
                for j, (col, cq) in enumerate(clause):
                    last = ci == len(spec) - 1 and j == len(clause) - 1
                    cnt = s.count if last else s.junk
                    if ci == 0:
                        qual_batched(cq, table(col), g.words, s.bitmap, cnt, stream=cs,
                                     or_src=s.bitmap if j else None)
                    elif len(clause) == 1:
                        qual_batched(cq, table(col), g.words, s.bitmap, cnt, stream=cs,
                                     and_dst=True)
                    elif j < len(clause) - 1:
                        qual_batched(cq, table(col), g.words, s.bm2, cnt, stream=cs,
                                     or_src=s.bm2 if j else None)
                    else:
                        qual_batched(cq, table(col), g.words, s.bitmap, cnt, stream=cs,
                                     or_src=s.bm2, and_dst=True)
            state["marks"].append((k, "quals_queued", time.perf_counter()))
            # emit tables: the strom_filter_batch prefix of the qual tables
            any_col = spec[0][0][0]
            d_rows = table(any_col)[:, :BATCH_FIELDS].contiguous()
            pstr = state.get("pchars") is not None
            d_proj = None
            if proj is not None:
                d_proj = table(proj) if pstr else table(proj)[:, :BATCH_FIELDS].contiguous()
            s.keep += [d_rows] + ([d_proj] if d_proj is not None else [])
        # decode + filter of successive groups overlap on their slots'
        # streams; the row-id emit (+ projection gather) runs in group order
        # on one stream (the output cursor is shared), and frees the slot
        ready = torch.cuda.Event()
        ready.record(cs)
        es = self.emit_stream
        es.wait_event(ready)
        with torch.cuda.stream(es):
            if pstr:
                bitmap_to_rows_str(s.bitmap, g.words, d_rows, state["out"], state["cursor"],
                                   d_proj, state["owidth"], state["poff"], state["pchars"],
                                   state["ccursor"], pvalid=state.get("pvalid"), stream=es)
            else:
                bitmap_to_rows(s.bitmap, g.words, d_rows, state["out"], state["cursor"],
                               stream=es, proj=d_proj, proj_out=state.get("pout"),
                               proj_valid=state.get("pvalid"))
            state["count"] += s.count
            s.count.zero_()
            if descs is not None:
                state["err"] += s.err
                s.err.zero_()
            s.event = torch.cuda.Event()
            s.event.record(es)
        state["bytes_read"] += g.read_bytes
        state["column_bytes"] += g.column_bytes
        state["marks"].append((k, "launched", time.perf_counter()))

    # ------------------------------------------------------------- query
    def dictionary(self, name: str):
        """Decoded dictionary of a dictionary-encoded column (host, cached):
        (values, valid) as utils.arrow_ipc.dictionary_values returns them."""
        if name not in self._dicts:
            col = self.meta.schema[self.meta.column_index(name)]
            self._dicts[name] = dictionary_values(self.meta, col, self.path)
        return self._dicts[name]

    def _compile(self, p: Pred) -> Compiled:
        key = (p.col, p.op, repr(p.value))
        if key not in self._compiled:
            col = self.meta.schema[self.meta.column_index(p.col)]
            dic = self.dictionary(p.col) if (col.dictionary is not None and
                                             p.op not in ("is_null", "is_valid")) else None
            self._compiled[key] = compile_pred(p, col, dic)
        return self._compiled[key]

    def scan_where(self, quals, project: Optional[str] = None,
                   batches: Optional[Tuple[int, int]] = None) -> ScanOut:
        """Row ids (int64, file order) of the rows every qualifier selects —
        a PG-Strom qualifier list.  ``quals`` items: ``(name, lo, hi)``
        ranges, ``(name, op, value)`` / ``P(name) <op> value`` predicates,
        or ``Or(...)`` clauses of them (ops/colpred.py: comparisons, IN,
        OR of ranges, string equality and prefix, null tests, on ints,
        floats, bool, date/time/timestamp/duration, utf8/binary and
        dictionary-encoded columns).  Nulls never satisfy a comparison.
        Each referenced column is read from storage and decoded once per
        group; the predicates' bitmaps are combined on the device.
        ``project`` names a column whose values (indices for a dictionary:
        ``ScanOut.dictionary`` holds the values; for utf8/binary the
        characters, with ``ScanOut.offsets``) and validity, when it has
        nulls, are gathered for the selected rows while their ids are
        written.  ``batches=(b0, b1)``
        scans only record batches [b0, b1) (row ids stay file-global:
        parallel/scan.py splits a file over ranks this way)."""
        cl = clauses(quals)
        t0 = time.perf_counter()
        names: List[str] = []
        for n in [p.col for c in cl for p in c] + ([project] if project else []):
            if n not in names:
                names.append(n)
        nb = self.meta.nbatches
        rng = (0, nb) if batches is None else (max(0, int(batches[0])), min(nb, int(batches[1])))
        key = (tuple(names), rng)
        if key not in self._plans:                # the file's layout is fixed once opened
            if tuple(names) not in self._bplans:
                self._bplans[tuple(names)] = self._plan(names)
            allb, cols, _ = self._bplans[tuple(names)]
            sel = allb[rng[0]:max(rng[0], rng[1])]
            self._plans[key] = (cols, int(sel.rows.sum()) if len(sel) else 0, self._groups(sel))
        cols, nrows, groups = self._plans[key]
        spec = [[(names.index(p.col), self._compile(p)) for p in c] for c in cl]
        t_plan = time.perf_counter()
        out = torch.empty(max(nrows, 1), dtype=torch.int64, device=self.device)
        pcol = names.index(project) if project else None
        pout = pvalid = pchars = poff = None
        pmeta = cols[pcol] if project else None
        pstrings = bool(project) and pmeta.kind in ("utf8", "binary") and pmeta.dictionary is None
        if project:
            st = pmeta.storage
            if pstrings:
                # characters: at most the column's, per the plan
                nch = sum(int(g.aux_len[:, pcol].sum()) for g in groups)
                pchars = torch.empty(max(nch, 1), dtype=torch.uint8, device=self.device)
                poff = torch.empty(max(nrows, 1) + 1, dtype=torch.int64, device=self.device)
            elif st == "d16":
                # decimal128: (lo, hi) int64 words per row, value x 10^scale
                pout = torch.empty((max(nrows, 1), 2), dtype=torch.int64, device=self.device)
            elif st not in _TORCH:
                raise NotImplementedError(f"projection of {project} ({pmeta.kind}): fixed-width, "
                                          "utf8/binary or dictionary-encoded columns")
            else:
                pout = torch.empty(max(nrows, 1), dtype=_TORCH[st], device=self.device)
            if any(bool(g.has_valid[pcol]) for g in groups):
                pvalid = torch.empty(max(nrows, 1), dtype=torch.uint8, device=self.device)
        pdict = self.dictionary(project) if project and pmeta.dictionary is not None else None
        if not groups or nrows == 0:
            return ScanOut(nrows, 0, out[:0], {"total_s": time.perf_counter() - t0},
                           values=pout[:0] if pout is not None else
                           (pchars[:0] if pchars is not None else None),
                           column=pmeta, dictionary=pdict,
                           offsets=torch.zeros(1, dtype=torch.int64, device=self.device)
                           if pstrings else None)
        self._ensure_slots(groups)
        # one emit stream per scan object (its library-kept scratch follows it)
        if getattr(self, "emit_stream", None) is None:
            self.emit_stream = torch.cuda.Stream(device=self.device)
        z = lambda: torch.zeros(1, dtype=torch.int64, device=self.device)
        state = dict(out=out, cursor=z(), count=z(), err=z(), wait_s=0.0, bytes_read=0,
                     column_bytes=0, pout=pout, pvalid=pvalid, pchars=pchars, poff=poff,
                     ccursor=z(), owidth=8 if pstrings and pmeta.large else 4, marks=[])
        t_alloc = time.perf_counter()
        # depth nslots - 1 of reads ahead of the group being computed
        ahead = max(1, min(self.nslots, len(self._slots)) - 1)
        for k in range(min(ahead, len(groups))):
            self._submit(k, groups[k])
            state["marks"].append((k, "submitted", time.perf_counter()))
        for k in range(len(groups)):
            self._compute(k, spec, pcol, state)
            if k + ahead < len(groups):
                self._submit(k + ahead, groups[k + ahead])
                state["marks"].append((k + ahead, "submitted", time.perf_counter()))
        torch.cuda.synchronize(self.device)
        cursor, count, err, nchars = torch.cat([state["cursor"], state["count"], state["err"],
                                                state["ccursor"]]).tolist()
        t_end = time.perf_counter()
        if err:
            raise RuntimeError(f"{'ZSTD' if self._codec == D.ARROW_ZSTD else 'LZ4'} decode "
                               f"failed for {err} buffer(s) of columns {names}")
        if cursor != count:
            raise RuntimeError(f"row emit mismatch: {cursor} ids for {count} selected")
        for s in self._slots:
            s.keep = []
            s.event = None
        offsets = None
        if pstrings:
            poff[count] = nchars
            offsets = poff[:count + 1]
        return ScanOut(nrows, int(count), out[:count],
                       {"plan_s": t_plan - t0, "alloc_s": t_alloc - t_plan,
                        "wait_s": state["wait_s"], "total_s": t_end - t0,
                        # per group: (group, event, ms since the scan's first submit)
                        "timeline_ms": [(k, e, round((t - t_alloc) * 1e3, 3))
                                        for k, e, t in state["marks"]]},
                       bytes_read=state["bytes_read"], column_bytes=state["column_bytes"],
                       groups=len(groups),
                       values=pout[:count] if pout is not None else
                       (pchars[:nchars] if pchars is not None else None),
                       valid=pvalid[:count] if pvalid is not None else None,
                       column=pmeta, dictionary=pdict, offsets=offsets)

    def scan(self, name: str, lo, hi) -> ScanOut:
        """Row ids (int64, file order) of ``lo <= column <= hi`` (nulls never
        qualify)."""
        return self.scan_where([(name, lo, hi)])

    # the pre-pipeline name
    filter = scan

    def host_scan_where(self, quals, project: Optional[str] = None,
                        batches: Optional[Tuple[int, int]] = None) -> "HostScanOut":
        """The same query on the CPU (buffers read with pread, decoded by
        the decoders' host twins, predicates by colpred's numpy twin)."""
        return host_scan_where(self.path, quals, project, batches, meta=self.meta,
                               dicts=self._dicts)

    def _free_slots(self) -> None:
        if self._slots:
            self._hbm.close()
        self._slots = []

    def close(self) -> None:
        self._free_slots()
        if self.reader is not None:
            self.reader.close()
            self.reader = None
        if getattr(self, "_pfd", None) is not None:
            os.close(self._pfd)
            self._pfd = None


# ------------------------------------------------------------ host twin
@dataclass
class HostScanOut:
    rows: int
    indices: np.ndarray                # int64 global row ids
    values: object = None              # projected values (numpy; strings: list of bytes)
    valid: Optional[np.ndarray] = None


def host_scan_where(path: str, quals, project: Optional[str] = None,
                    batches: Optional[Tuple[int, int]] = None, meta: Optional[ArrowFile] = None,
                    dicts: Optional[dict] = None) -> HostScanOut:
    """ArrowScan.scan_where on the CPU: the same metadata, the same
    compiled predicates (ops/colpred.py), evaluated by the kernel's numpy
    twin over buffers decoded by the GPU decoders' host twins.  The
    reference point for the GPU path and a scan for machines without one."""
    meta = meta if meta is not None else read_metadata(path)
    dicts = dicts if dicts is not None else {}
    cl = clauses(quals)
    schema = {c.name: (i, c) for i, c in enumerate(meta.schema)}

    def dictionary(name):
        if name not in dicts:
            dicts[name] = dictionary_values(meta, schema[name][1], path)
        return dicts[name]
    comp = []
    for c in cl:
        row = []
        for p in c:
            col = schema[p.col][1]
            dic = dictionary(p.col) if col.dictionary is not None and \
                p.op not in ("is_null", "is_valid") else None
            row.append((p.col, compile_pred(p, col, dic)))
        comp.append(row)
    names = sorted({n for c in comp for n, _ in c} | ({project} if project else set()))
    nb = meta.nbatches
    b0, b1 = (0, nb) if batches is None else (max(0, batches[0]), min(nb, batches[1]))
    base = np.concatenate([[0], np.cumsum(meta.rows)]).astype(np.int64)
    ids, vals, valid = [], [], []
    src = _Src(path)
    try:
        for bi in range(b0, b1):
            b = meta.batches[bi]
            data = {}
            for n in names:
                ci, col = schema[n]
                ch = b.columns[ci]
                vraw = read_buffer(src, ch.validity, b.codec) if ch.null_count else b""
                d = read_buffer(src, ch.data, b.codec)
                vcol = col if col.dictionary is None else Column(n, "int", col.dictionary.index_bits,
                                                                 col.dictionary.index_signed)
                x = read_buffer(src, ch.extra, b.codec) if (ch.extra is not None and
                                                            col.dictionary is None) else b""
                data[n] = (decode_values(vcol, ch.length, d, x), validity_bits(vraw, ch.length))
            n = b.length
            m = np.ones(n, bool)
            for c in comp:
                cm = np.zeros(n, bool)
                for name, cq in c:
                    v, ok = data[name]
                    cm |= evaluate(cq, v, ok, n)
                m &= cm
            sel = np.flatnonzero(m)
            ids.append(sel + base[bi])
            if project:
                v, ok = data[project]
                if isinstance(v, tuple):
                    offs, chars = v
                    vals.append([chars[offs[i]:offs[i + 1]].tobytes() for i in sel])
                else:
                    vals.append(np.asarray(v)[sel])
                valid.append(ok[sel] if ok is not None else np.ones(len(sel), bool))
    finally:
        src.close()
    out = HostScanOut(int(base[b1] - base[b0]) if b1 > b0 else 0,
                      np.concatenate(ids) if ids else np.zeros(0, np.int64))
    if project:
        if vals and isinstance(vals[0], list):
            out.values = [x for v in vals for x in v]
        else:
            out.values = np.concatenate(vals) if vals else np.zeros(0)
        vv = np.concatenate(valid) if valid else np.zeros(0, bool)
        out.valid = None if vv.all() else vv
    return out
