"""PostgreSQL heap tuples with real tuple descriptors: builder + host deformer.

The GPU heap scanner's general mode (``strom_heap_scan2``,
csrc/kernels/heapscan.hip) deforms tuples the way PostgreSQL's
``slot_deform_heap_tuple`` does and evaluates a qualifier list over them —
what the reference gets by handing every tuple to ``ExecScan``
(pgsql/nvme_strom.c:1137-1143, tuple walk :1054-1092).  This module is its
host-side twin and test oracle, written from PostgreSQL's on-disk rules, not
from the kernel:

* ``TupleDesc``: attlen / attalign per column from PostgreSQL type names
  (pg_type: int2 's', int4 'i', int8 / float8 / timestamp 'd', text 'i' ...);
* ``heap_tuple``: ``heap_fill_tuple``'s layout — null bitmap (t_bits) when
  any attribute is NULL, attalign padding, varlenas converted to 1-byte
  short headers when they fit (<= 126 data bytes), else aligned 4-byte
  headers; ``Toast`` / ``Compressed`` values write a TOAST pointer
  (va_tag VARTAG_ONDISK) or a compressed inline datum;
* ``deform``: the attribute walk (``att_align_pointer``: a varlena is
  aligned only when the byte at the current offset is a pad byte);
* ``host_scan2``: items + per-page status of a scan with a qualifier list,
  the reference result the GPU must equal.

No PostgreSQL server exists here: parity with a live server is unpinned.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from decimal import Decimal, localcontext
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np

from . import pgpage

# name -> (attlen, attalign, value kind)
PG_TYPES = {
    "bool": (1, 1, "int"), "char": (1, 1, "int"), "int2": (2, 2, "int"),
    "int4": (4, 4, "int"), "int8": (8, 8, "int"), "oid": (4, 4, "int"),
    "date": (4, 4, "int"), "time": (8, 8, "int"), "timestamp": (8, 8, "int"),
    "timestamptz": (8, 8, "int"), "float4": (4, 4, "float"), "float8": (8, 8, "float"),
    "text": (-1, 4, "text"), "varchar": (-1, 4, "text"), "bpchar": (-1, 4, "text"),
    "bytea": (-1, 4, "text"), "numeric": (-1, 4, "numeric"), "jsonb": (-1, 4, "text"),
    "name": (64, 1, "bytes"), "cstring": (-2, 1, "text"),
}

HEAP_HASNULL = 0x0001
VARTAG_ONDISK = 18
PAGE_RECHECK = 8


class Toast:
    """An out-of-line value: the tuple holds an 18-byte TOAST pointer."""

    def __init__(self, valueid: int = 1):
        self.valueid = valueid


class Compressed:
    """An inline compressed value (4-byte header with the compressed bit)."""

    def __init__(self, payload: bytes = b"\x00" * 12):
        self.payload = payload


EXT = object()   # deform's marker for a compressed / out-of-line varlena


def _align(off: int, al: int) -> int:
    return (off + al - 1) & ~(al - 1)


@dataclass
class TupleDesc:
    names: List[str]
    types: List[str]
    attlen: List[int] = field(init=False)
    attalign: List[int] = field(init=False)
    kinds: List[str] = field(init=False)

    def __post_init__(self):
        if len(self.names) != len(self.types):
            raise ValueError("names and types differ in length")
        self.attlen = [PG_TYPES[t][0] for t in self.types]
        self.attalign = [PG_TYPES[t][1] for t in self.types]
        self.kinds = [PG_TYPES[t][2] for t in self.types]

    @classmethod
    def of(cls, cols: Sequence[Tuple[str, str]]) -> "TupleDesc":
        return cls([c[0] for c in cols], [c[1] for c in cols])

    @property
    def natts(self) -> int:
        return len(self.names)

    def attno(self, col) -> int:
        return col if isinstance(col, int) else self.names.index(col)

    def cacheoff(self) -> List[int]:
        """attcacheoff: the offset after t_hoff of each fixed-length attribute
        whose predecessors are all fixed-length (valid for null-free
        tuples), else -1."""
        out, off, fixed = [], 0, True
        for L, al in zip(self.attlen, self.attalign):
            if fixed and L > 0:
                off = _align(off, al)
                out.append(off)
                off += L
            else:
                out.append(-1)
                fixed = False
        return out


# ---- numeric (src/backend/utils/adt/numeric.c on-disk form): base-10000
# digits, NumericShort when the display scale and weight fit, else
# NumericLong; NaN / +-Infinity as special headers
NBASE = 10000


def numeric_parts(v) -> Tuple[int, int, int, List[int], int]:
    """(kind 0 finite / 1 NaN / 2 +inf / 3 -inf, negative, weight, digits,
    dscale) of a Decimal / int / float / str, digits with no leading or
    trailing zero groups (zero: no digits, weight 0)."""
    d = v if isinstance(v, Decimal) else Decimal(str(v))
    if d.is_nan():
        return 1, 0, 0, [], 0
    if d.is_infinite():
        return (2 if d > 0 else 3), 0, 0, [], 0
    sign, digits, exp = d.as_tuple()
    dscale = max(0, -exp)
    coef = int("".join(map(str, digits))) if digits else 0
    k = (dscale + 3) // 4
    n = coef * 10 ** (4 * k + exp)
    groups: List[int] = []
    while n:
        groups.insert(0, n % NBASE)
        n //= NBASE
    if not groups:
        return 0, 0, 0, [], dscale
    weight = len(groups) - 1 - k
    while groups and groups[-1] == 0:
        groups.pop()
    return 0, int(sign), weight, groups, dscale


def numeric_bytes(v) -> bytes:
    """The numeric's varlena payload (without the varlena header)."""
    kind, neg, weight, digits, dscale = numeric_parts(v)
    if kind:
        return struct.pack("<H", {1: 0xC000, 2: 0xD000, 3: 0xF000}[kind])
    body = struct.pack(f"<{len(digits)}h", *digits)
    if dscale <= 0x3F and -64 <= weight <= 63:
        h = 0x8000 | (0x2000 if neg else 0) | (dscale << 7) | (0x40 if weight < 0 else 0) | \
            (weight & 0x3F)
        return struct.pack("<H", h) + body
    return struct.pack("<Hh", (0x4000 if neg else 0) | (dscale & 0x3FFF), weight) + body


def numeric_value(raw: bytes) -> Decimal:
    """A numeric's varlena payload back to a Decimal."""
    h, = struct.unpack_from("<H", raw, 0)
    if h & 0xC000 == 0xC000:
        sp = h & 0xF000
        return Decimal({0xC000: "NaN", 0xD000: "Infinity", 0xF000: "-Infinity"}[sp])
    if h & 0xC000 == 0x8000:
        neg = bool(h & 0x2000)
        weight = (h | ~0x3F) if h & 0x40 else h & 0x3F
        body = raw[2:]
    else:
        neg = (h & 0xC000) == 0x4000
        weight, = struct.unpack_from("<h", raw, 2)
        body = raw[4:]
    digits = struct.unpack(f"<{len(body) // 2}h", body[:len(body) // 2 * 2])
    with localcontext() as ctx:
        ctx.prec = 4 * len(digits) + 8
        val = sum((Decimal(d) * (Decimal(NBASE) ** (weight - i)) for i, d in enumerate(digits)),
                  Decimal(0))
        return -val if neg else +val


def numeric_key(v) -> Tuple[int, Decimal]:
    """PostgreSQL's numeric order: -inf < finite < +inf < NaN (NaN = NaN)."""
    d = v if isinstance(v, Decimal) else Decimal(str(v))
    if d.is_nan():
        return (3, Decimal(0))
    if d.is_infinite():
        return (2 if d > 0 else 0, Decimal(0))
    return (1, d)


def _datum(v: Any, L: int, kind: str, al: int, off: int) -> Tuple[int, bytes]:
    """(aligned offset, bytes) of a non-null attribute stored at ``off``."""
    if L > 0:
        off = _align(off, al)
        if kind == "float":
            b = struct.pack("<f" if L == 4 else "<d", float(v))
        elif kind == "bytes":
            raw = v.encode() if isinstance(v, str) else bytes(v)
            b = raw[:L].ljust(L, b"\0")
        else:
            b = int(v).to_bytes(L, "little", signed=True)
        return off, b
    if L == -2:
        raw = v.encode() if isinstance(v, str) else bytes(v)
        return off, raw + b"\0"
    if isinstance(v, Toast):
        # 1-byte header 0x01, vartag, varatt_external {rawsize, extinfo, valueid, toastrelid}
        return off, bytes([1, VARTAG_ONDISK]) + struct.pack("<iIII", 100, 96, v.valueid, 16384)
    if isinstance(v, Compressed):
        off = _align(off, al)
        n = 4 + 4 + len(v.payload)
        return off, struct.pack("<I", (n << 2) | 2) + struct.pack("<I", 1000) + v.payload
    if kind == "numeric":
        raw = numeric_bytes(v)
    else:
        raw = v.encode() if isinstance(v, str) else bytes(v)
    if len(raw) + 1 <= 0x7F:                 # VARATT_CAN_MAKE_SHORT: no alignment
        return off, bytes([((len(raw) + 1) << 1) | 1]) + raw
    off = _align(off, al)
    return off, struct.pack("<I", (len(raw) + 4) << 2) + raw


def heap_tuple(values: Sequence[Any], desc: TupleDesc, infomask: int = pgpage.VISIBLE,
               natts: Optional[int] = None, xmin: int = 2, xmax: int = 0) -> bytes:
    """A tuple as heap_form_tuple lays it out; ``natts`` < len(values) keeps
    only the first attributes (a row written before ALTER TABLE ADD COLUMN)."""
    n = desc.natts if natts is None else natts
    vals = list(values)[:n]
    hasnull = any(v is None for v in vals)
    nbitmap = (n + 7) // 8 if hasnull else 0
    hoff = pgpage.maxalign(23 + nbitmap)
    data = bytearray()
    bits = bytearray(nbitmap)
    for i, v in enumerate(vals):
        if v is None:
            continue
        if hasnull:
            bits[i >> 3] |= 1 << (i & 7)
        off, b = _datum(v, desc.attlen[i], desc.kinds[i], desc.attalign[i], len(data))
        data += b"\0" * (off - len(data)) + b
    mask = infomask | (HEAP_HASNULL if hasnull else 0)
    hdr = struct.pack("<IIIHHHHHB", xmin, xmax, 0, 0, 0, 0, n & 0x7FF, mask, hoff)
    return hdr + bytes(bits) + b"\0" * (hoff - 23 - nbitmap) + bytes(data)


def build_pages(rows: Sequence[Sequence[Any]], desc: TupleDesc, page_sz: int = 8192,
                with_checksum: bool = True, natts_of=None, blkno_base: int = 0) -> bytes:
    """Pack tuples into as few pages as fit (``natts_of(i)`` the stored
    attribute count of row i)."""
    pages, cur, used = [], [], pgpage.SIZE_OF_PAGE_HEADER
    for i, r in enumerate(rows):
        t = heap_tuple(r, desc, natts=natts_of(i) if natts_of else None)
        need = pgpage.maxalign(len(t)) + 4
        if cur and used + need > page_sz:
            pages.append(pgpage.build_page(cur, blkno_base + len(pages), page_sz, with_checksum))
            cur, used = [], pgpage.SIZE_OF_PAGE_HEADER
        cur.append(t)
        used += need
    if cur:
        pages.append(pgpage.build_page(cur, blkno_base + len(pages), page_sz, with_checksum))
    return b"".join(pages)


def deform(tup: bytes, desc: TupleDesc) -> List[Any]:
    """Attribute values of a tuple (None for NULL / not stored, EXT for a
    compressed or out-of-line varlena); raises ValueError when malformed."""
    infomask2, infomask = struct.unpack_from("<HH", tup, 18)
    hoff = tup[22]
    natts = infomask2 & 0x7FF
    hasnull = bool(infomask & HEAP_HASNULL)
    out, off = [], hoff
    for i in range(desc.natts):
        if i >= natts or (hasnull and not (tup[23 + (i >> 3)] >> (i & 7)) & 1):
            out.append(None)
            continue
        L, al, kind = desc.attlen[i], desc.attalign[i], desc.kinds[i]
        if L > 0:
            off = _align(off, al)
            raw = tup[off:off + L]
            if len(raw) < L:
                raise ValueError("attribute past the tuple end")
            if kind == "float":
                out.append(struct.unpack("<f" if L == 4 else "<d", raw)[0])
            elif kind == "bytes":
                out.append(bytes(raw))
            else:
                out.append(int.from_bytes(raw, "little", signed=True))
            off += L
        elif L == -1:
            if tup[off] == 0:                       # pad byte: aligned 4-byte header
                off = _align(off, al)
            b = tup[off]
            if b & 1 == 0:
                n = (struct.unpack_from("<I", tup, off)[0] >> 2) & 0x3FFFFFFF
                out.append(EXT if b & 3 == 2 else bytes(tup[off + 4:off + n]))
            elif b == 1:
                n = 2 + {18: 16, 1: 8, 2: 8, 3: 8}[tup[off + 1]]
                out.append(EXT)
            else:
                n = b >> 1
                out.append(bytes(tup[off + 1:off + n]))
            if kind == "numeric" and out[-1] is not EXT:
                out[-1] = numeric_value(out[-1])
            if off + n > len(tup):
                raise ValueError("varlena past the tuple end")
            off += n
        else:
            e = tup.index(b"\0", off)
            out.append(bytes(tup[off:e]))
            off = e + 1
    return out


def _b(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


@dataclass
class Qual:
    """One qualifier over column ``col`` (name or 0-based attno): ``op`` in
    between (inclusive) / eq / lt / le / gt / ge / in / isnull / notnull on
    int, float and numeric columns; text_eq / prefix / text_in on varlena
    text.  A qualifier list is ANDed; ``Or(...)`` groups qualifiers into one
    ORed clause (conjunctive normal form)."""
    col: Any
    op: str
    args: tuple = ()

    def test(self, v: Any, kind: str) -> Optional[bool]:
        """True / False, or None when undecidable (EXT under a text or
        numeric op)."""
        if self.op == "isnull":
            return v is None
        if v is None:
            return False
        if self.op == "notnull":
            return True
        if self.op in ("text_eq", "prefix", "text_in"):
            if v is EXT:
                return None
            if self.op == "text_in":
                return v in {_b(c) for c in self.args[0]}
            c = _b(self.args[0])
            return v == c if self.op == "text_eq" else v.startswith(c)
        if kind == "numeric":
            if self.op == "in" and not self.args[0]:
                return False                     # constant false, whatever v is
            if v is EXT:
                return None
            k = numeric_key(v)
            if self.op == "in":
                return any(k == numeric_key(c) for c in self.args[0])
            if self.op == "between":
                return numeric_key(self.args[0]) <= k <= numeric_key(self.args[1])
            c = numeric_key(self.args[0])
            return {"eq": k == c, "lt": k < c, "le": k <= c, "gt": k > c, "ge": k >= c}[self.op]
        if self.op in ("lt", "le", "gt", "ge"):
            c = self.args[0]
            if kind == "float":
                return {"lt": not _pg_le(c, v), "le": _pg_le(v, c), "gt": not _pg_le(v, c),
                        "ge": _pg_le(c, v)}[self.op]
            return {"lt": v < c, "le": v <= c, "gt": v > c, "ge": v >= c}[self.op]
        if self.op == "between":
            lo, hi = self.args
            if kind == "float":
                return _pg_le(float(lo), v) and _pg_le(v, float(hi))
            return lo <= v <= hi
        if self.op == "eq":
            return v == self.args[0] if kind != "float" else (_pg_le(self.args[0], v) and _pg_le(v, self.args[0]))
        if self.op == "in":
            if kind == "float":
                return any(_pg_le(c, v) and _pg_le(v, c) for c in self.args[0])
            return v in self.args[0]
        raise ValueError(self.op)


class Or:
    """An ORed clause of qualifiers in a qualifier list (CNF)."""

    def __init__(self, *quals: Qual):
        if not quals:
            raise ValueError("empty Or")
        self.quals = list(quals)

    def __repr__(self) -> str:
        return "Or(" + ", ".join(map(repr, self.quals)) + ")"


def clauses(quals) -> List[List[Qual]]:
    """A qualifier list as CNF clauses (each a list of ORed Quals)."""
    return [q.quals if isinstance(q, Or) else [q] for q in quals]


def _pg_le(x: float, y: float) -> bool:
    if y != y:
        return True
    if x != x:
        return False
    return x <= y


def host_scan2(data: bytes, desc: TupleDesc, quals: Sequence[Qual], page_sz: int = 8192,
               skip_invisible: bool = False, verify_checksum: bool = False,
               blkno_base: int = 0, project=None) -> Tuple[List[int], List[int], list]:
    """Reference scan with a qualifier list: (sorted item ids page<<16|lineno,
    per-page status incl. PAGE_RECHECK, projected values of the items: one
    value per item, a tuple of values when ``project`` lists columns)."""
    items, status, proj = [], [], []
    many = isinstance(project, (list, tuple))
    pj = ([desc.attno(c) for c in project] if many else
          desc.attno(project) if project is not None else None)
    for pg in range(len(data) // page_sz):
        page = data[pg * page_sz:(pg + 1) * page_sz]
        _, st = pgpage.host_scan(page, page_sz, False, verify_checksum=verify_checksum,
                                 blkno_base=blkno_base + pg)
        st = st[0]
        if st:
            status.append(st)
            continue
        _, flags, lower = struct.unpack_from("<HHH", page, 8)
        found = []
        for i in range((lower - 24) // 4):
            lp, = struct.unpack_from("<I", page, 24 + 4 * i)
            off, fl, ln = lp & 0x7FFF, (lp >> 15) & 3, lp >> 17
            if fl != pgpage.LP_NORMAL or ln < 23 or off < 24 or off + ln > page_sz or off & 1:
                continue
            tup = page[off:off + ln]
            infomask, = struct.unpack_from("<H", tup, 20)
            if skip_invisible and not pgpage.tuple_visible(infomask, flags):
                continue
            try:
                vals = deform(tup, desc)
            except (ValueError, KeyError, IndexError):
                continue
            # CNF, three-valued: a clause is true if any of its quals is,
            # unknown if none is but one is undecidable (EXT), else false
            verdict = True
            for cl in clauses(quals):
                cv = False
                for q in cl:
                    k = desc.attno(q.col)
                    r = q.test(vals[k], desc.kinds[k])
                    if r is True:
                        cv = True
                        break
                    if r is None:
                        cv = None
                if cv is False:
                    verdict = False
                    break
                if cv is None:
                    verdict = None
            if verdict is None:
                st |= PAGE_RECHECK
            elif verdict:
                found.append((i + 1, tuple(vals[k] for k in pj) if many else
                              vals[pj] if pj is not None else None))
        status.append(st)
        for lineno, v in found:
            items.append((pg << 16) | lineno)
            proj.append(v)
    order = np.argsort(np.array(items, dtype=np.int64), kind="stable") if items else []
    return [items[j] for j in order], status, [proj[j] for j in order]


def synthetic(n: int, seed: int = 0) -> Tuple[TupleDesc, list]:
    """A 10-column relation for benches: NULLs in most columns, short and
    long text before the numeric columns, TOAST pointers and compressed
    datums in ``note``."""
    desc = TupleDesc.of([("id", "int4"), ("name", "text"), ("a", "int8"), ("flag", "bool"),
                         ("b", "float8"), ("note", "text"), ("c", "int2"), ("d", "date"),
                         ("e", "float4"), ("tail", "int8")])
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        name = None if rng.random() < 0.15 else (
            f"k{int(rng.integers(0, 40))}" if rng.random() < 0.9 else "L" * int(rng.integers(127, 300)))
        r = rng.random()
        note = (None if r < 0.2 else Toast(i) if r < 0.25 else Compressed() if r < 0.3
                else "ab" + "x" * int(rng.integers(0, 20)) if r < 0.6 else "zz" * int(rng.integers(1, 90)))
        rows.append([i, name, None if rng.random() < 0.1 else int(rng.integers(-10**6, 10**6)),
                     int(rng.random() < 0.5), None if rng.random() < 0.1 else float(rng.random()),
                     note, int(rng.integers(-5, 6)), int(rng.integers(0, 20000)),
                     None if rng.random() < 0.05 else float(rng.normal()),
                     int(rng.integers(-100, 100))])
    return desc, rows
