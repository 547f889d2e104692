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
class ArrowFile:
    schema: List[Column]
    batches: List[Batch]
    size: int

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
        hit = self._cache.pop((off, n), None) if hasattr(self, "_cache") else None
        if hit is not None:
            return hit
        import os
        return os.pread(self.fd, n, off)

    def prefetch(self, ranges, threads: int = 16) -> None:
        """Read many small ranges at once: a file's record-batch headers sit
        between the bodies, one small read each, which on a cold file cost
        one storage round trip apiece when read in sequence (the cold-scan
        cost of an Arrow file with thousands of batches)."""
        if self.buf is not None or len(ranges) < 8:
            return
        import os
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=threads) as ex:
            got = list(ex.map(lambda r: os.pread(self.fd, r[1], r[0]), ranges))
        self._cache = dict(zip(ranges, got))

    def close(self):
        if self.fd is not None:
            import os
            os.close(self.fd)


def read_metadata(path_or_bytes) -> ArrowFile:
    src = _Src(path_or_bytes)
    try:
        return _read(src)
    finally:
        src.close()


def _read(src: "_Src") -> ArrowFile:
    if src.read(0, 6) != MAGIC or src.read(src.size - 6, 6) != MAGIC:
        raise ValueError("not an Arrow IPC file")
    flen, = struct.unpack("<i", src.read(src.size - 10, 4))
    fbuf = src.read(src.size - 10 - flen, flen)
    footer = FB.root(fbuf, 0)
    schema_fb = footer.table(1)
    schema = [_column(f) for f in schema_fb.tables(1)] if schema_fb else []
    start, n = footer.vector(3)
    batches = []
    src.prefetch([tuple(struct.unpack_from("<qi", fbuf, start + 24 * k)) for k in range(n)])
    for k in range(n):
        boff, mlen, blen = struct.unpack_from("<qi4xq", fbuf, start + 24 * k)
        buf = src.read(boff, mlen)
        msg, _ = _message(buf, 0)
        htype = msg.scalar(1, "B", 0)
        if htype != 3:
            continue
        rb = msg.table(2)
        body = boff + mlen
        comp = rb.table(3)
        codec = None
        if comp is not None:
            codec = {0: "lz4_frame", 1: "zstd"}.get(comp.scalar(0, "b", 0), "unknown")
        nstart, nn = rb.vector(1)
        nodes = [struct.unpack_from("<qq", buf, nstart + 16 * i) for i in range(nn)]
        bstart, bn = rb.vector(2)
        bufs = [struct.unpack_from("<qq", buf, bstart + 16 * i) for i in range(bn)]
        b = Batch(boff, rb.scalar(0, "q", 0), body, blen, codec)
        cursor = [0, 0]                     # next node, next buffer

        def walk(col: Column) -> Optional[ColumnChunk]:
            if col.nbuffers < 0:
                raise ValueError(f"column {col.name}: layout not supported")
            ni, bi = cursor
            ln, nc = nodes[ni]
            own = bufs[bi:bi + col.nbuffers]
            cursor[0] += 1
            cursor[1] += col.nbuffers
            for ch in col.children:
                walk(ch)
            if col.nbuffers == 2:
                (vo, vl), (do, dl) = own
                return ColumnChunk(ln, nc, BufferRef(body + vo, vl), BufferRef(body + do, dl))
            return ColumnChunk(ln, nc, BufferRef(0, 0), BufferRef(0, 0))

        for col in schema:
            b.columns.append(walk(col))
        batches.append(b)
    return ArrowFile(schema, batches, src.size)
