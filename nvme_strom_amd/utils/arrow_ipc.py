"""Minimal Apache Arrow IPC *file* reader: metadata only, no data decoding.

The scan path needs the byte ranges of each record batch's buffers inside
the file (to load them into HBM with the engine and decode them on the GPU),
not an Arrow library doing the reads and decompression on the CPU.  This
module walks the flatbuffer metadata (File.fbs Footer/Block, Message.fbs
Message/RecordBatch/FieldNode/Buffer/BodyCompression, Schema.fbs
Schema/Field/Int/FloatingPoint) with a ~60-line flatbuffer reader.

Supported columns: fixed-width primitives (int8..64, uint8..64, float16/32/64)
— the kinds the GPU filter evaluates.  Other columns are listed with
``supported = False``.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

MAGIC = b"ARROW1"


# --------------------------------------------------------------- flatbuffers
class FB:
    def __init__(self, buf: bytes, pos: int):
        self.buf = buf
        self.pos = pos
        vt = pos - struct.unpack_from("<i", buf, pos)[0]
        self.vt = vt
        self.vt_len = struct.unpack_from("<H", buf, vt)[0]

    @staticmethod
    def root(buf: bytes, off: int = 0) -> "FB":
        return FB(buf, off + struct.unpack_from("<I", buf, off)[0])

    def _field(self, i: int) -> int:
        o = 4 + 2 * i
        if o >= self.vt_len:
            return 0
        return struct.unpack_from("<H", self.buf, self.vt + o)[0]

    def scalar(self, i: int, fmt: str, default=0):
        f = self._field(i)
        return struct.unpack_from("<" + fmt, self.buf, self.pos + f)[0] if f else default

    def _ref(self, i: int) -> Optional[int]:
        f = self._field(i)
        if not f:
            return None
        p = self.pos + f
        return p + struct.unpack_from("<I", self.buf, p)[0]

    def table(self, i: int) -> Optional["FB"]:
        p = self._ref(i)
        return FB(self.buf, p) if p is not None else None

    def vector(self, i: int) -> Tuple[int, int]:
        """(element start, length)"""
        p = self._ref(i)
        if p is None:
            return 0, 0
        return p + 4, struct.unpack_from("<I", self.buf, p)[0]

    def tables(self, i: int) -> List["FB"]:
        start, n = self.vector(i)
        out = []
        for k in range(n):
            e = start + 4 * k
            out.append(FB(self.buf, e + struct.unpack_from("<I", self.buf, e)[0]))
        return out

    def string(self, i: int) -> str:
        start, n = self.vector(i)
        return self.buf[start:start + n].decode() if n else ""


# ------------------------------------------------------------------ schema
@dataclass
class Column:
    name: str
    kind: str                  # "int" | "float" | "other"
    bit_width: int = 0
    signed: bool = True
    nullable: bool = True
    nbuffers: int = 2          # own buffers (validity + data for primitives)
    children: List["Column"] = field(default_factory=list)
    supported: bool = True     # the GPU filter can evaluate it

    @property
    def numpy_dtype(self) -> str:
        if self.kind == "int":
            return f"{'i' if self.signed else 'u'}{self.bit_width // 8}"
        return {16: "f2", 32: "f4", 64: "f8"}[self.bit_width]


_TYPE_INT, _TYPE_FP = 2, 3
# own buffer count per Schema.fbs Type id (None = layout not walkable here)
_NBUF = {1: 0, 2: 2, 3: 2, 4: 3, 5: 3, 6: 2, 7: 2, 8: 2, 9: 2, 10: 2, 11: 2, 12: 2, 13: 1,
         15: 2, 16: 1, 17: 2, 18: 2, 19: 3, 20: 3, 21: 2}


def _column(f: FB) -> Column:
    name = f.string(0)
    nullable = bool(f.scalar(1, "B", 0))
    ttype = f.scalar(2, "B", 0)
    t = f.table(3)
    children = [_column(c) for c in f.tables(5)]
    if ttype == _TYPE_INT and t is not None:
        return Column(name, "int", t.scalar(0, "i", 0), bool(t.scalar(1, "B", 0)), nullable)
    if ttype == _TYPE_FP and t is not None:
        prec = t.scalar(0, "h", 0)
        return Column(name, "float", {0: 16, 1: 32, 2: 64}[prec], True, nullable)
    return Column(name, "other", nullable=nullable, nbuffers=_NBUF.get(ttype, -1),
                  children=children, supported=False)


# ----------------------------------------------------------------- batches
@dataclass
class BufferRef:
    offset: int                # absolute file offset
    length: int                # bytes in the file (compressed incl. 8-B prefix)


@dataclass
class ColumnChunk:
    length: int
    null_count: int
    validity: BufferRef
    data: BufferRef


@dataclass
class Batch:
    offset: int                # message start in the file
    length: int                # rows
    body_offset: int
    body_length: int
    codec: Optional[str]       # None | "lz4_frame" | "zstd"
    columns: List[ColumnChunk] = field(default_factory=list)


@dataclass
class ColumnArrays:
    """One column's chunks over all record batches, as arrays (batch order)."""
    length: np.ndarray
    null_count: np.ndarray
    v_off: np.ndarray          # validity buffer: absolute file offset, stored bytes
    v_len: np.ndarray
    d_off: np.ndarray          # data buffer
    d_len: np.ndarray


class ArrowFile:
    """Schema + record-batch layout.  The layout is held as arrays
    (``rows``, ``codecs``, ``columns[i]``: ColumnArrays); ``batches`` builds
    the per-batch objects on first use (a scan plan reads the arrays)."""

    def __init__(self, schema: List[Column], size: int, offset=None, rows=None, body=None,
                 body_len=None, codecs=None, columns=None):
        self.schema = schema
        self.size = size
        z = np.zeros(0, np.int64)
        self.offset = offset if offset is not None else z
        self.rows = rows if rows is not None else z
        self.body = body if body is not None else z
        self.body_len = body_len if body_len is not None else z
        self.codecs: List[Optional[str]] = codecs if codecs is not None else []
        self.columns: List[ColumnArrays] = columns if columns is not None else []
        self._batches: Optional[List[Batch]] = None

    @property
    def nbatches(self) -> int:
        return len(self.rows)

    @property
    def batches(self) -> List[Batch]:
        if self._batches is None:
            percol = []
            for c in self.columns:
                it = zip(*(a.tolist() for a in (c.length, c.null_count, c.v_off, c.v_len,
                                                 c.d_off, c.d_len)))
                percol.append([ColumnChunk(a, b, BufferRef(vo, vl), BufferRef(do, dl))
                               for a, b, vo, vl, do, dl in it])
            self._batches = [
                Batch(o, r, bo, bl, cd, [c[j] for c in percol])
                for j, (o, r, bo, bl, cd) in enumerate(zip(
                    self.offset.tolist(), self.rows.tolist(), self.body.tolist(),
                    self.body_len.tolist(), self.codecs))]
        return self._batches

    def __eq__(self, other) -> bool:
        return (isinstance(other, ArrowFile) and self.schema == other.schema
                and self.size == other.size and self.batches == other.batches)

    def column_index(self, name: str) -> int:
        for i, c in enumerate(self.schema):
            if c.name == name:
                return i
        raise KeyError(name)


def _message(buf: bytes, off: int) -> Tuple[FB, int]:
    cont, = struct.unpack_from("<i", buf, off)
    if cont == -1:
        mlen, = struct.unpack_from("<i", buf, off + 4)
        return FB.root(buf, off + 8), off + 8 + mlen
    # legacy: no continuation marker
    return FB.root(buf, off + 4), off + 4 + cont


class _Src:
    """Byte source: an in-memory buffer or a file read with pread (only the
    footer and the message headers are ever read, never the bodies)."""

    def __init__(self, path_or_bytes):
        if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
            self.buf, self.fd = bytes(path_or_bytes), None
            self.size = len(self.buf)
        else:
            import os
            self.buf, self.fd = None, os.open(path_or_bytes, os.O_RDONLY)
            self.size = os.fstat(self.fd).st_size

    def read(self, off: int, n: int) -> bytes:
        if self.buf is not None:
            return self.buf[off:off + n]
        import os
        return os.pread(self.fd, n, off)

    def close(self):
        if self.fd is not None:
            import os
            os.close(self.fd)


def read_metadata(path_or_bytes, native: Optional[bool] = None) -> ArrowFile:
    """Schema and record-batch layout of an Arrow IPC file.  For a file path
    the record-batch headers are read and parsed by libstrom
    (csrc/engine/arrow_meta.cc: many reads in flight, no per-header Python);
    ``native=False`` (or an in-memory source) takes the Python walk below."""
    src = _Src(path_or_bytes)
    try:
        return _read(src, native if native is not None else src.fd is not None)
    finally:
        src.close()


def _layout(schema: List[Column]) -> Tuple[List[Tuple[int, int, int]], int, int]:
    """(first node, first buffer, own buffers) of every top-level column:
    the same in every record batch (children follow their parent)."""
    cur = [0, 0]

    def walk(col: Column):
        if col.nbuffers < 0:
            raise ValueError(f"column {col.name}: layout not supported")
        me = (cur[0], cur[1], col.nbuffers)
        cur[0] += 1
        cur[1] += col.nbuffers
        for ch in col.children:
            walk(ch)
        return me

    return [walk(c) for c in schema], cur[0], cur[1]


_CODECS = {-1: None, 0: "lz4_frame", 1: "zstd"}


def _headers_py(src: "_Src", blocks: np.ndarray, nn: int, nb: int):
    """Python reference of strom_arrow_headers: the same output arrays."""
    n = len(blocks)
    rows = np.zeros(n, np.int64)
    codec = np.zeros(n, np.int32)
    nodes = np.zeros((n, nn, 2), np.int64)
    bufs = np.zeros((n, nb, 2), np.int64)
    for k, (boff, mlen, _) in enumerate(blocks.tolist()):
        buf = src.read(boff, mlen)
        msg, _ = _message(buf, 0)
        if msg.scalar(1, "B", 0) != 3:
            codec[k] = -2
            continue
        rb = msg.table(2)
        comp = rb.table(3)
        codec[k] = -1 if comp is None else comp.scalar(0, "b", 0)
        rows[k] = rb.scalar(0, "q", 0)
        for vi, arr, cap in ((1, nodes, nn), (2, bufs, nb)):
            start, cnt = rb.vector(vi)
            if cnt < cap:
                raise ValueError(f"record batch {k}: {cnt} entries, schema needs {cap}")
            arr[k] = np.frombuffer(buf, "<i8", 2 * cap, start).reshape(cap, 2)
    return rows, codec, nodes, bufs


def _headers_native(src: "_Src", blocks: np.ndarray, nn: int, nb: int, threads: int = 32):
    import ctypes as C

    from .. import _native
    n = len(blocks)
    mx_n, mx_b = nn + 64, nb + 128          # room for trailing entries the schema walk ignores
    rows = np.zeros(n, np.int64)
    codec = np.zeros(n, np.int32)
    cn = np.zeros(n, np.int32)
    cb = np.zeros(n, np.int32)
    nodes = np.zeros((n, mx_n, 2), np.int64)
    bufs = np.zeros((n, mx_b, 2), np.int64)
    bad = np.full(1, -1, np.int64)
    blk = np.ascontiguousarray(blocks, dtype=np.int64)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    rc = _native.lib().strom_arrow_headers(src.fd, p(blk), n, mx_n, mx_b, p(rows), p(codec),
                                           p(cn), p(cb), p(nodes), p(bufs), threads, p(bad))
    if rc != 0:
        raise ValueError(f"Arrow record-batch headers: rc={rc}, first bad block {int(bad[0])}")
    ok = codec == -2
    short = ~ok & ((cn < nn) | (cb < nb))
    if short.any():
        k = int(np.flatnonzero(short)[0])
        raise ValueError(f"record batch {k}: {cn[k]}/{cb[k]} entries, schema needs {nn}/{nb}")
    return rows, codec, nodes[:, :nn], bufs[:, :nb]


def _read(src: "_Src", native: bool = False) -> ArrowFile:
    if src.read(0, 6) != MAGIC or src.read(src.size - 6, 6) != MAGIC:
        raise ValueError("not an Arrow IPC file")
    flen, = struct.unpack("<i", src.read(src.size - 10, 4))
    fbuf = src.read(src.size - 10 - flen, flen)
    footer = FB.root(fbuf, 0)
    schema_fb = footer.table(1)
    schema = [_column(f) for f in schema_fb.tables(1)] if schema_fb else []
    start, n = footer.vector(3)
    # Block structs: offset i64, metaDataLength i32 (+4 pad), bodyLength i64
    raw = np.frombuffer(fbuf, np.dtype([("off", "<i8"), ("mlen", "<i4"), ("pad", "<i4"),
                                        ("blen", "<i8")]), n, start)
    blocks = np.stack([raw["off"], raw["mlen"].astype(np.int64), raw["blen"]], axis=1)
    if n == 0:
        return ArrowFile(schema, src.size)
    lay, nn, nb = _layout(schema)
    rows, codec, nodes, bufs = (_headers_native if native else _headers_py)(src, blocks, nn, nb)
    body = blocks[:, 0] + blocks[:, 1]
    keep = np.flatnonzero(codec != -2)
    names = {c: _CODECS.get(c, "unknown") for c in set(codec[keep].tolist())}
    bo = body[keep]
    cols = []
    for ni, bi, own in lay:
        z = np.zeros(len(keep), np.int64)
        if own == 2:
            cols.append(ColumnArrays(nodes[keep, ni, 0], nodes[keep, ni, 1],
                                     bo + bufs[keep, bi, 0], bufs[keep, bi, 1],
                                     bo + bufs[keep, bi + 1, 0], bufs[keep, bi + 1, 1]))
        else:
            cols.append(ColumnArrays(nodes[keep, ni, 0], nodes[keep, ni, 1], z, z, z, z))
    return ArrowFile(schema, src.size, blocks[keep, 0], rows[keep], bo, blocks[keep, 2],
                     [names[c] for c in codec[keep].tolist()], cols)
