"""Minimal Apache Arrow IPC *file* reader: metadata only, no data decoding.

The scan path needs the byte ranges of each record batch's buffers inside
the file (to load them into HBM with the engine and decode them on the GPU),
not an Arrow library doing the reads and decompression on the CPU.  This
module walks the flatbuffer metadata (File.fbs Footer/Block, Message.fbs
Message/RecordBatch/FieldNode/Buffer/BodyCompression, Schema.fbs
Schema/Field/Int/FloatingPoint) with a ~60-line flatbuffer reader.

Scan-able columns (``supported``): fixed-width integers and floats,
bool (bit-packed), date32/64, time32/64, timestamp (any unit, tz kept),
duration, utf8/binary and their large (64-bit offset) forms, and
dictionary-encoded columns of those (the record batches carry the index
column; the dictionaries come from the file's DictionaryBatch messages,
Message.fbs DictionaryBatch{id, data, isDelta}, and are decoded on the
host: they are small and a predicate on one becomes a lookup table over
the indices).  Other columns (decimal, nested, views) are listed with
``supported = False``; a file holding a variadic-buffer view column cannot
be laid out and is refused.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

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
class DictEncoding:
    """Schema.fbs DictionaryEncoding: the record batches hold ``index``
    integers into dictionary ``id`` (Int indexType, int32 when absent)."""
    id: int
    index_bits: int = 32
    index_signed: bool = True
    ordered: bool = False


@dataclass
class Column:
    name: str
    kind: str                  # int float bool date time timestamp duration utf8 binary other
    bit_width: int = 0         # fixed-width value bits (the date/time/... storage integer)
    signed: bool = True
    nullable: bool = True
    nbuffers: int = 2          # own buffers (validity + data for primitives)
    children: List["Column"] = field(default_factory=list)
    supported: bool = True     # the GPU scan can evaluate predicates on it
    unit: str = ""             # date: "d"/"ms"; time/timestamp/duration: "s" "ms" "us" "ns"
    tz: str = ""               # timestamp time zone ("" = naive)
    large: bool = False        # utf8/binary with 64-bit offsets
    dictionary: Optional[DictEncoding] = None
    precision: int = 0         # decimal: digits, and the power of ten the stored integer
    scale: int = 0             # is divided by

    @property
    def storage(self) -> str:
        """numpy dtype of the record-batch data buffer: the value integers
        or floats, the offsets of a utf8/binary column, the indices of a
        dictionary-encoded one; "b1" for bit-packed bools."""
        if self.dictionary is not None:
            d = self.dictionary
            return f"{'i' if d.index_signed else 'u'}{d.index_bits // 8}"
        if self.kind in ("utf8", "binary"):
            return "i8" if self.large else "i4"
        if self.kind == "bool":
            return "b1"
        if self.kind == "decimal":
            return "d16"       # 128-bit two's complement, little-endian
        if self.kind == "float":
            return {16: "f2", 32: "f4", 64: "f8"}[self.bit_width]
        if self.kind in _INTLIKE:
            return f"{'i' if self.signed else 'u'}{self.bit_width // 8}"
        raise ValueError(f"column {self.name}: no storage type for {self.kind}")

    @property
    def numpy_dtype(self) -> str:
        return self.storage


_INTLIKE = ("int", "date", "time", "timestamp", "duration")
# Schema.fbs Type union ids
(_TY_INT, _TY_FP, _TY_BIN, _TY_UTF8, _TY_BOOL, _TY_DEC, _TY_DATE, _TY_TIME, _TY_TS, _TY_DUR,
 _TY_LBIN, _TY_LUTF8) = 2, 3, 4, 5, 6, 7, 8, 9, 10, 18, 19, 20
_TUNIT = ("s", "ms", "us", "ns")       # TimeUnit enum
# own buffer count per Schema.fbs Type id (None = layout not walkable here)
_NBUF = {1: 0, 2: 2, 3: 2, 4: 3, 5: 3, 6: 2, 7: 2, 8: 2, 9: 2, 10: 2, 11: 2, 12: 2, 13: 1,
         15: 2, 16: 1, 17: 2, 18: 2, 19: 3, 20: 3, 21: 2}


def _value_type(name: str, nullable: bool, ttype: int, t: Optional[FB]) -> Column:
    """The Column of a Schema.fbs type table (flatbuffer defaults applied:
    writers omit fields equal to them — Date.unit MILLISECOND, Time.unit
    MILLISECOND + bitWidth 32, Duration.unit MILLISECOND)."""
    g = (lambda i, fmt, d: t.scalar(i, fmt, d)) if t is not None else (lambda i, fmt, d: d)
    if ttype == _TY_INT and t is not None:
        return Column(name, "int", g(0, "i", 0), bool(g(1, "B", 0)), nullable)
    if ttype == _TY_FP and t is not None:
        bits = {0: 16, 1: 32, 2: 64}[g(0, "h", 0)]
        return Column(name, "float", bits, True, nullable, supported=bits != 16)
    if ttype == _TY_BOOL:
        return Column(name, "bool", 1, False, nullable)
    if ttype == _TY_DEC:
        # Decimal{precision, scale, bitWidth = 128}: decimal128 is scanned,
        # decimal256 listed only
        bits = g(2, "i", 128)
        return Column(name, "decimal", bits, True, nullable, supported=bits == 128,
                      precision=g(0, "i", 0), scale=g(1, "i", 0))
    if ttype in (_TY_UTF8, _TY_LUTF8, _TY_BIN, _TY_LBIN):
        return Column(name, "utf8" if ttype in (_TY_UTF8, _TY_LUTF8) else "binary", 0, False,
                      nullable, nbuffers=3, large=ttype in (_TY_LBIN, _TY_LUTF8))
    if ttype == _TY_DATE:
        day = g(0, "h", 1) == 0
        return Column(name, "date", 32 if day else 64, True, nullable, unit="d" if day else "ms")
    if ttype == _TY_TIME:
        return Column(name, "time", g(1, "i", 32), True, nullable, unit=_TUNIT[g(0, "h", 1)])
    if ttype == _TY_TS:
        return Column(name, "timestamp", 64, True, nullable, unit=_TUNIT[g(0, "h", 0)],
                      tz=t.string(1) if t is not None else "")
    if ttype == _TY_DUR:
        return Column(name, "duration", 64, True, nullable, unit=_TUNIT[g(0, "h", 1)])
    return Column(name, "other", nullable=nullable, nbuffers=_NBUF.get(ttype, -1),
                  supported=False)


def _column(f: FB) -> Column:
    name = f.string(0)
    nullable = bool(f.scalar(1, "B", 0))
    col = _value_type(name, nullable, f.scalar(2, "B", 0), f.table(3))
    de = f.table(4)
    if de is not None:
        # dictionary-encoded: one node + validity/index buffers in the
        # record batches whatever the value type (its children, if any,
        # live in the dictionary batches)
        it = de.table(1)
        col.dictionary = DictEncoding(de.scalar(0, "q", 0),
                                      it.scalar(0, "i", 32) if it is not None else 32,
                                      bool(it.scalar(1, "B", 1)) if it is not None else True,
                                      bool(de.scalar(2, "B", 0)))
        col.supported = col.kind != "other"
        col.nbuffers = 2
        return col
    if col.kind == "other":
        col.children = [_column(c) for c in f.tables(5)]
    return col


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
    data: BufferRef            # values / indices / utf8-binary offsets
    extra: Optional[BufferRef] = None   # utf8/binary: the character data


@dataclass
class DictBatch:
    """One DictionaryBatch message: the value column's node and buffers
    (absolute file offsets), in the order the value type lays them out."""
    id: int
    length: int
    null_count: int
    codec: Optional[str]
    buffers: List[BufferRef]
    delta: bool


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
    x_off: Optional[np.ndarray] = None   # third buffer (utf8/binary data)
    x_len: Optional[np.ndarray] = None


class ArrowFile:
    """Schema + record-batch layout.  The layout is held as arrays
    (``rows``, ``codecs``, ``columns[i]``: ColumnArrays); ``batches`` builds
    the per-batch objects on first use (a scan plan reads the arrays)."""

    def __init__(self, schema: List[Column], size: int, offset=None, rows=None, body=None,
                 body_len=None, codecs=None, columns=None, dicts=None):
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
        # dictionary id -> its DictionaryBatch messages in file order
        self.dicts: Dict[int, List[DictBatch]] = dicts if dicts is not None else {}

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
                ch = [ColumnChunk(a, b, BufferRef(vo, vl), BufferRef(do, dl))
                      for a, b, vo, vl, do, dl in it]
                if c.x_off is not None:
                    for k, (xo, xl) in enumerate(zip(c.x_off.tolist(), c.x_len.tolist())):
                        ch[k].extra = BufferRef(xo, xl)
                percol.append(ch)
            self._batches = [
                Batch(o, r, bo, bl, cd, [c[j] for c in percol])
                for j, (o, r, bo, bl, cd) in enumerate(zip(
                    self.offset.tolist(), self.rows.tolist(), self.body.tolist(),
                    self.body_len.tolist(), self.codecs))]
        return self._batches

    def __eq__(self, other) -> bool:
        return (isinstance(other, ArrowFile) and self.schema == other.schema
                and self.size == other.size and self.batches == other.batches
                and self.dicts == other.dicts)

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
        if own in (2, 3):
            ca = ColumnArrays(nodes[keep, ni, 0], nodes[keep, ni, 1],
                              bo + bufs[keep, bi, 0], bufs[keep, bi, 1],
                              bo + bufs[keep, bi + 1, 0], bufs[keep, bi + 1, 1])
            if own == 3:
                ca.x_off, ca.x_len = bo + bufs[keep, bi + 2, 0], bufs[keep, bi + 2, 1]
            cols.append(ca)
        else:
            cols.append(ColumnArrays(nodes[keep, ni, 0], nodes[keep, ni, 1], z, z, z, z))
    return ArrowFile(schema, src.size, blocks[keep, 0], rows[keep], bo, blocks[keep, 2],
                     [names[c] for c in codec[keep].tolist()], cols,
                     _dictionaries(src, footer, fbuf))


def _dictionaries(src: "_Src", footer: FB, fbuf: bytes) -> Dict[int, List[DictBatch]]:
    """Footer.dictionaries -> DictionaryBatch messages (Message.fbs
    header_type 2: DictionaryBatch{id, data: RecordBatch, isDelta}).  Only
    their headers are read here; values are decoded when a scan needs them.
    The file is input data: a malformed header is a ValueError."""
    try:
        return _dictionaries_walk(src, footer, fbuf)
    except (struct.error, IndexError, UnicodeDecodeError) as e:
        raise ValueError(f"malformed dictionary batch header: {e}") from None


def _dictionaries_walk(src: "_Src", footer: FB, fbuf: bytes) -> Dict[int, List[DictBatch]]:
    start, n = footer.vector(2)
    out: Dict[int, List[DictBatch]] = {}
    for k in range(n):
        boff, mlen, _, _ = struct.unpack_from("<qiiq", fbuf, start + 24 * k)
        buf = src.read(boff, mlen)
        msg, _ = _message(buf, 0)
        if msg.scalar(1, "B", 0) != 2:
            raise ValueError(f"dictionary block {k}: not a DictionaryBatch message")
        db = msg.table(2)
        rb = db.table(1) if db is not None else None
        if rb is None:
            raise ValueError(f"dictionary block {k}: no data")
        comp = rb.table(3)
        codec = _CODECS.get(-1 if comp is None else comp.scalar(0, "b", 0), "unknown")
        ns, nn = rb.vector(1)
        bs, nb = rb.vector(2)
        length, nulls = (struct.unpack_from("<qq", buf, ns) if nn else (0, 0))
        base = boff + mlen
        bufs = [BufferRef(base + o, ln) for o, ln in
                (struct.unpack_from("<qq", buf, bs + 16 * j) for j in range(nb))]
        did = db.scalar(0, "q", 0)
        out.setdefault(did, []).append(DictBatch(did, rb.scalar(0, "q", length), nulls, codec,
                                                 bufs, bool(db.scalar(2, "B", 0))))
    return out


# ------------------------------------------------------------ host decode
def read_buffer(src, ref: BufferRef, codec: Optional[str]) -> bytes:
    """One stored buffer, decompressed on the host (Arrow BodyCompression:
    i64 uncompressed length, -1 = stored raw, then the frame).  The host
    twins of the GPU decoders do the work (ops/decompress.py), so the file's
    codecs need no CPU library.  ``src``: a path, bytes or an open _Src."""
    own = not isinstance(src, _Src)
    s = _Src(src) if own else src
    try:
        raw = s.read(ref.offset, ref.length)
    finally:
        if own:
            s.close()
    if codec is None or not raw:
        return raw
    n, = struct.unpack_from("<q", raw, 0)
    if n == -1:
        return raw[8:]
    from ..ops import decompress as D
    if codec == "zstd":
        st, out = D.zstd_host(D.ARROW_ZSTD, raw, n)
    elif codec == "lz4_frame":
        st, out, _ = D.lz4par_host(D.ARROW_LZ4, raw, n)
    else:
        raise ValueError(f"body compression {codec}")
    if st != n:
        raise ValueError(f"buffer at {ref.offset}: decoded {st} of {n} bytes")
    return out


def validity_bits(raw: bytes, n: int) -> Optional[np.ndarray]:
    """Arrow LSB-first validity bytes -> bool[n] (None: all valid)."""
    if not raw:
        return None
    return np.unpackbits(np.frombuffer(raw, np.uint8), bitorder="little")[:n].astype(bool)


def decode_values(col: Column, length: int, data: bytes, extra: bytes = b""):
    """A chunk's values as numpy: fixed-width -> the storage dtype array;
    bool -> bool array; utf8/binary -> (int64 offsets[length + 1], uint8
    data).  (For a dictionary-encoded column ``col`` describes the VALUE
    type and ``data``/``extra`` are the dictionary's buffers.)"""
    if col.kind == "bool":
        return np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[:length].astype(bool)
    if col.kind in ("utf8", "binary"):
        offs = np.frombuffer(data, "<i8" if col.large else "<i4", length + 1) if length else \
            np.zeros(1, np.int64)
        return offs.astype(np.int64), np.frombuffer(extra, np.uint8)
    if col.kind == "decimal":
        # the stored 128-bit integers (value x 10^scale) as Python ints
        return np.array([int.from_bytes(data[16 * i:16 * i + 16], "little", signed=True)
                         for i in range(length)], dtype=object)
    dt = np.dtype("<" + (Column(col.name, col.kind, col.bit_width, col.signed).storage))
    return np.frombuffer(data, dt, length)


def dictionary_values(meta: "ArrowFile", col: Column, src) -> Tuple[object, Optional[np.ndarray]]:
    """The decoded dictionary of a dictionary-encoded column: (values,
    valid) with values as decode_values returns them, deltas appended in
    file order.  Two non-delta batches for one id (a replacement) are
    refused: the file format does not allow them."""
    if col.dictionary is None:
        raise ValueError(f"column {col.name} is not dictionary-encoded")
    parts = meta.dicts.get(col.dictionary.id, [])
    if not parts:
        raise ValueError(f"column {col.name}: dictionary {col.dictionary.id} missing")
    if any(not p.delta for p in parts[1:]):
        raise ValueError(f"column {col.name}: dictionary replaced inside an IPC file")
    vals, valid, strings = [], [], col.kind in ("utf8", "binary")
    for p in parts:
        need = 3 if strings else 2
        if len(p.buffers) < need:
            raise ValueError(f"dictionary {p.id}: {len(p.buffers)} buffers")
        bufs = [read_buffer(src, b, p.codec) for b in p.buffers[:need]]
        v = decode_values(col, p.length, bufs[1], bufs[2] if strings else b"")
        vals.append(v)
        vb = validity_bits(bufs[0], p.length) if p.null_count else None
        valid.append(vb if vb is not None else np.ones(p.length, bool))
    if strings:
        offs, datas, base = [np.zeros(1, np.int64)], [], 0
        for o, d in vals:
            offs.append(o[1:] - o[0] + base)
            datas.append(d[o[0]:o[-1]])
            base += int(o[-1] - o[0])
        out = (np.concatenate(offs), np.concatenate(datas) if datas else np.zeros(0, np.uint8))
    else:
        out = np.concatenate(vals)
    vv = np.concatenate(valid)
    return out, (None if vv.all() else vv)
