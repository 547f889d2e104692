"""Arrow scan predicates: the forms a query writes, their compilation to the
operands of the GPU qualifier kernel (csrc/kernels/colfilter.hip,
``strom_column_qual``), and a numpy twin of that kernel.

A qualifier list is a conjunction (CNF): each item is one predicate or an
``Or`` of predicates (on any columns).  Predicates:

    (name, lo, hi)                      lo <= v <= hi (the round-1 form)
    (name, op, value)  /  P(name) <op> value
        "==" "!=" "<" "<=" ">" ">="     numeric, bool, date/time/timestamp/duration,
                                        utf8/binary (bytewise, as pyarrow)
        "between" (lo, hi)              inclusive
        "in" / "not in" [values]        IN-lists (numbers, strings, dates ...)
        "ranges" [(lo, hi), ...]        an OR of inclusive ranges on one column
        "prefix" / "not prefix" s       utf8/binary starts-with (a list: any of)
    (name, "is_null") / (name, "is_valid")

Nulls never satisfy a comparison (SQL: a NULL comparison is not true, and
NOT of it is not true either), so every predicate's bits are ANDed with the
row's validity; ``Or`` of a NULL and a true predicate is true.  Floats
follow pyarrow.compute: NaN compares false (so ``!=`` selects it) and
``in`` matches NaN to a NaN in the list.  Integers compare exactly (bounds
in the column's own integer domain: ``v < 2.5`` is ``v <= 2``), floats in
double (pyarrow promotes float32 against a Python float the same way).

Dictionary-encoded columns are evaluated on the dictionary (host, numpy,
this module's twin) and the GPU tests each row's index against the
resulting lookup table — any predicate, including string ranges, costs one
bit test per row.  The reference has no columnar path (new
MI355X work); the predicate model follows PG-Strom's qualifier lists.
"""
from __future__ import annotations

import ctypes as C
import datetime as _dt
import math
import struct
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from ..utils.arrow_ipc import Column

# strom.h: STROM_COL_* storage types, STROM_QOP_* operators, STROM_QUAL_* flags
COL_CODE = {"i4": 1, "i8": 2, "f4": 3, "f8": 4, "i1": 5, "i2": 6, "u1": 7, "u2": 8, "u4": 9,
            "u8": 10, "b1": 11, "d16": 14}
COL_STR32, COL_STR64 = 12, 13
QOP_RANGES, QOP_STR_IN, QOP_STR_PREFIX, QOP_LUT, QOP_VALID, QOP_STR_RANGES = 1, 2, 3, 4, 5, 6
FLAG_NEGATE, FLAG_NAN = 1, 2
MAX_RANGES = 4096                 # the kernel stages constants in LDS (<= 64 KiB)
MAX_CONST_BYTES = 48 << 10
MAX_LUT_BITS = 512 << 10

OPS = {"==", "!=", "<", "<=", ">", ">=", "between", "in", "not in", "ranges", "prefix",
       "not prefix", "is_null", "is_valid"}
_NEG = {"!=": "==", "not in": "in", "not prefix": "prefix"}


@dataclass(frozen=True)
class Pred:
    col: str
    op: str
    value: object = None

    def __post_init__(self):
        if self.op not in OPS:
            raise ValueError(f"predicate op {self.op!r}: one of {sorted(OPS)}")


class P:
    """Builder: ``P("name") == "abc"``, ``P("d").between(a, b)``,
    ``P("k").isin([1, 5])``, ``P("s").startswith("ab")``."""

    def __init__(self, col: str):
        self.col = col

    def __eq__(self, v): return Pred(self.col, "==", v)      # noqa: E704
    def __ne__(self, v): return Pred(self.col, "!=", v)      # noqa: E704
    def __lt__(self, v): return Pred(self.col, "<", v)       # noqa: E704
    def __le__(self, v): return Pred(self.col, "<=", v)      # noqa: E704
    def __gt__(self, v): return Pred(self.col, ">", v)       # noqa: E704
    def __ge__(self, v): return Pred(self.col, ">=", v)      # noqa: E704
    __hash__ = None

    def between(self, lo, hi) -> Pred:
        return Pred(self.col, "between", (lo, hi))

    def isin(self, values) -> Pred:
        return Pred(self.col, "in", tuple(values))

    def not_in(self, values) -> Pred:
        return Pred(self.col, "not in", tuple(values))

    def ranges(self, rs) -> Pred:
        return Pred(self.col, "ranges", tuple(tuple(r) for r in rs))

    def startswith(self, prefix) -> Pred:
        return Pred(self.col, "prefix", prefix)

    def is_null(self) -> Pred:
        return Pred(self.col, "is_null")

    def is_valid(self) -> Pred:
        return Pred(self.col, "is_valid")


@dataclass(frozen=True)
class Or:
    preds: Tuple[Pred, ...]

    def __init__(self, *preds):
        object.__setattr__(self, "preds", tuple(as_pred(p) for p in preds))
        if not self.preds:
            raise ValueError("Or() of nothing")


def as_pred(q) -> Pred:
    if isinstance(q, Pred):
        return q
    if isinstance(q, tuple) and len(q) >= 2 and isinstance(q[0], str):
        if isinstance(q[1], str) and q[1] in OPS:
            return Pred(q[0], q[1], q[2] if len(q) > 2 else None)
        if len(q) == 3:
            return Pred(q[0], "between", (q[1], q[2]))
    raise ValueError(f"not a predicate: {q!r}")


def clauses(quals) -> List[List[Pred]]:
    """CNF: a list of OR-clauses (each a list of predicates), ANDed."""
    out = []
    for q in quals:
        if isinstance(q, Or):
            out.append(list(q.preds))
        elif isinstance(q, list):
            out.append([as_pred(p) for p in q])
        else:
            out.append([as_pred(q)])
    if not out:
        raise ValueError("at least one qualifier")
    return out


# ------------------------------------------------------------ compilation
@dataclass
class Compiled:
    """Kernel operands of one predicate on one column's record-batch data."""
    type: int                       # STROM_COL_*
    op: int                         # STROM_QOP_*
    flags: int = 0
    nconst: int = 0
    consts: bytes = b""             # ranges / string blob / LUT words
    offs: bytes = b""               # strings: (start, len) uint32 pairs
    # numpy twin operands
    ranges: Optional[np.ndarray] = None       # (n, 2) in the compare domain
    strings: Optional[List[bytes]] = None
    lut: Optional[np.ndarray] = None          # bool per dictionary index
    _dev: Dict[str, object] = field(default_factory=dict, repr=False)


_TICKS = {"s": 1, "ms": 10 ** 3, "us": 10 ** 6, "ns": 10 ** 9}
_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)


def _exact(v, col: Column) -> Fraction:
    """A scalar as an exact rational in the column's storage domain
    (date32 days, date64 ms, time/timestamp/duration ticks of its unit)."""
    if isinstance(v, (bool, np.bool_)):
        return Fraction(int(v))
    if isinstance(v, (int, np.integer)):
        return Fraction(int(v))
    if isinstance(v, Fraction):
        return v
    if isinstance(v, (float, np.floating)):
        if math.isnan(v) or math.isinf(v):
            raise OverflowError
        return Fraction(float(v))
    import decimal as _dec
    if isinstance(v, _dec.Decimal):
        if not v.is_finite():
            raise OverflowError
        return Fraction(v)
    k = col.kind
    tick = Fraction(86400) if col.unit == "d" else Fraction(1, _TICKS.get(col.unit, 1))
    if hasattr(v, "to_datetime64") or hasattr(v, "to_timedelta64"):   # pandas scalars
        v = v.to_datetime64() if hasattr(v, "to_datetime64") else v.to_timedelta64()
    if isinstance(v, np.datetime64) or isinstance(v, np.timedelta64):
        ns = int(v.astype("datetime64[ns]" if isinstance(v, np.datetime64)
                          else "timedelta64[ns]").astype(np.int64))
        return Fraction(ns, 10 ** 9) / tick
    if isinstance(v, str) and k in ("date", "timestamp"):
        v = (_dt.date.fromisoformat(v) if k == "date" and len(v) == 10
             else _dt.datetime.fromisoformat(v))
    if isinstance(v, _dt.datetime):
        if v.tzinfo is None:
            v = v.replace(tzinfo=_dt.timezone.utc)
        d = v - _EPOCH
        secs = Fraction(d.days * 86400 + d.seconds) + Fraction(d.microseconds, 10 ** 6)
        return secs / tick
    if isinstance(v, _dt.date):
        return Fraction((v - _dt.date(1970, 1, 1)).days * 86400) / tick
    if isinstance(v, _dt.time):
        secs = Fraction(v.hour * 3600 + v.minute * 60 + v.second) + Fraction(v.microsecond, 10 ** 6)
        return secs / tick
    if isinstance(v, _dt.timedelta):
        secs = Fraction(v.days * 86400 + v.seconds) + Fraction(v.microseconds, 10 ** 6)
        return secs / tick
    raise TypeError(f"column {col.name} ({col.kind}): cannot compare with {type(v).__name__}")


def _int_bounds(dt: str) -> Tuple[int, int]:
    if dt == "b1":
        return 0, 1
    if dt == "d16":
        return -(1 << 127), (1 << 127) - 1
    info = np.iinfo(np.dtype(dt))
    return int(info.min), int(info.max)


def _dbl(v, col: Column) -> float:
    if isinstance(v, (float, np.floating)):
        return float(v)
    return float(_exact(v, col))


def _dbl_floor(x: Fraction) -> float:
    f = float(x)
    return f if Fraction(f) <= x else math.nextafter(f, -math.inf)


def _dbl_ceil(x: Fraction) -> float:
    f = float(x)
    return f if Fraction(f) >= x else math.nextafter(f, math.inf)


def _merge(rs: List[Tuple], adjacent_int: bool) -> List[Tuple]:
    rs = sorted(r for r in rs if r[0] <= r[1])
    out: List[list] = []
    for lo, hi in rs:
        if out and lo <= out[-1][1] + (1 if adjacent_int else 0):
            out[-1][1] = max(out[-1][1], hi)
        else:
            out.append([lo, hi])
    return [tuple(r) for r in out]


def _dec_float_bound(x: float, side: str, scale: Fraction, tmin: int, tmax: int) -> int:
    """Bound on the unscaled integer u of a decimal column compared with a
    float constant the way pyarrow.compute does it: the column is cast to
    float64, so u qualifies iff float64(u / 10^scale) <op> x (float() of a
    Fraction rounds correctly, as the cast does for |u| < 2^53).  That map
    is monotone in u, so the bound is the first u whose float passes
    (``>=`` / ``>``), or the one before it (``<`` / ``<=``), found by
    bisection over the storage range (float spacing can exceed 10^-scale,
    so several u round onto x)."""
    strict = side in (">", "<=")               # first u with fl(u) > x, else >= x

    def ok(u: int) -> bool:
        f = float(Fraction(u) / scale)
        return f > x if strict else f >= x
    lo, hi = tmin - 1, tmax + 1                # ok(lo) taken false, ok(hi) true
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if ok(mid):
            hi = mid
        else:
            lo = mid
    return hi if side in (">", ">=") else hi - 1


def _num_ranges(op: str, v, col: Column, dt: str) -> Tuple[List[Tuple], int]:
    """(ranges in the compare domain, extra flags) of a numeric predicate
    (op already stripped of its negation)."""
    isf = dt in ("f4", "f8")
    if isf:
        def bound(x, side):                   # side: "<", "<=", ">", ">="
            if isinstance(x, (float, np.floating)) and math.isnan(x):
                return None
            if isinstance(x, (float, np.floating)) and math.isinf(x):
                f = float(x)
            else:
                e = _exact(x, col)
                f = _dbl_floor(e) if side in ("<", "<=") else _dbl_ceil(e)
                if side == "<" and Fraction(f) == e:
                    f = math.nextafter(f, -math.inf)
                if side == ">" and Fraction(f) == e:
                    f = math.nextafter(f, math.inf)
                return f
            if side == "<":
                return math.nextafter(f, -math.inf)
            if side == ">":
                return math.nextafter(f, math.inf)
            return f
        NEG, POS = -math.inf, math.inf
    else:
        tmin, tmax = _int_bounds(dt)

        scale = Fraction(10) ** col.scale if col.kind == "decimal" else 1

        def bound(x, side):
            if col.kind == "decimal" and isinstance(x, (float, np.floating)) and math.isfinite(x):
                return _dec_float_bound(float(x), side, scale, tmin, tmax)
            try:
                e = _exact(x, col) * scale
            except OverflowError:               # NaN compares false, +-inf past any int
                if isinstance(x, (float, np.floating)) and math.isinf(x):
                    return tmax + 1 if x > 0 else tmin - 1
                return None
            if side == "<":
                return math.ceil(e) - 1
            if side == "<=":
                return math.floor(e)
            if side == ">":
                return math.floor(e) + 1
            return math.ceil(e)
        NEG, POS = tmin, tmax

    def rng(lo_v, lo_side, hi_v, hi_side):
        lo = NEG if lo_v is None else bound(lo_v, lo_side)
        hi = POS if hi_v is None else bound(hi_v, hi_side)
        if lo is None or hi is None:
            return []
        if not isf:
            lo, hi = max(lo, tmin), min(hi, tmax)
        return [(lo, hi)] if lo <= hi else []

    flags = 0
    if op == "==":
        rs = rng(v, ">=", v, "<=")
    elif op == "<":
        rs = rng(None, "", v, "<")
    elif op == "<=":
        rs = rng(None, "", v, "<=")
    elif op == ">":
        rs = rng(v, ">", None, "")
    elif op == ">=":
        rs = rng(v, ">=", None, "")
    elif op == "between":
        lo, hi = v
        rs = rng(lo, ">=", hi, "<=")
    elif op in ("in", "ranges"):
        rs = []
        for x in v:
            if op == "in":
                if isf and isinstance(x, (float, np.floating)) and math.isnan(x):
                    flags |= FLAG_NAN
                    continue
                rs += rng(x, ">=", x, "<=")
            else:
                rs += rng(x[0], ">=", x[1], "<=")
    else:
        raise ValueError(f"column {col.name} ({col.kind}): op {op!r} not defined")
    return _merge(rs, not isf), flags


def _string_const(v, col: Column) -> bytes:
    if isinstance(v, str):
        return v.encode()
    if isinstance(v, (bytes, bytearray, memoryview, np.bytes_)):
        return bytes(v)
    raise TypeError(f"column {col.name} ({col.kind}): cannot compare with {type(v).__name__}")


def _string_ranges(op: str, v, col: Column, code: int, flags: int) -> Compiled:
    """Bytewise-lexicographic ranges (pyarrow compares utf8 by its bytes):
    per range two bounds (start, len, mode), mode 0 unbounded, 1
    inclusive, 2 exclusive."""
    sc = lambda x: _string_const(x, col)
    if op == "<":
        rs = [(None, 0, sc(v), 2)]
    elif op == "<=":
        rs = [(None, 0, sc(v), 1)]
    elif op == ">":
        rs = [(sc(v), 2, None, 0)]
    elif op == ">=":
        rs = [(sc(v), 1, None, 0)]
    elif op == "between":
        rs = [(sc(v[0]), 1, sc(v[1]), 1)]
    elif op == "ranges":
        rs = [(sc(a), 1, sc(b), 1) for a, b in v]
    else:
        raise ValueError(f"column {col.name} ({col.kind}): op {op!r} not defined")
    blob, offs = bytearray(), []
    for lo, lm, hi, hm in rs:
        for b, m in ((lo, lm), (hi, hm)):
            b = b or b""
            offs += [len(blob), len(b), m]
            blob += b + b"\0" * (-len(b) % 4)
    if len(blob) > MAX_CONST_BYTES or len(rs) > MAX_RANGES:
        raise ValueError(f"column {col.name}: {len(rs)} string ranges, {len(blob)} bytes")
    return Compiled(code, QOP_STR_RANGES, flags, len(rs), bytes(blob) or b"\0\0\0\0",
                    np.asarray(offs, np.uint32).tobytes(), strings=rs)


def _compile_value(p: Pred, col: Column, dt: str, code: int) -> Compiled:
    """A predicate on a plain (not dictionary-encoded) column."""
    op = p.op
    neg = op in _NEG
    base = _NEG.get(op, op)
    if base in ("is_null", "is_valid"):
        return Compiled(code, QOP_VALID, FLAG_NEGATE if base == "is_null" else 0)
    flags = FLAG_NEGATE if neg else 0
    if col.kind in ("utf8", "binary"):
        if base == "==":
            vals, qop = [_string_const(p.value, col)], QOP_STR_IN
        elif base == "in":
            vals, qop = [_string_const(x, col) for x in p.value], QOP_STR_IN
        elif base == "prefix":
            pv = p.value if isinstance(p.value, (list, tuple)) else [p.value]
            vals, qop = [_string_const(x, col) for x in pv], QOP_STR_PREFIX
        else:
            return _string_ranges(base, p.value, col, code, flags)
        vals = sorted(set(vals))
        blob, offs = bytearray(), []
        for b in vals:
            offs += [len(blob), len(b)]
            blob += b + b"\0" * (-len(b) % 4)
        if len(blob) > MAX_CONST_BYTES or len(vals) > MAX_RANGES:
            raise ValueError(f"column {col.name}: {len(vals)} string constants, "
                             f"{len(blob)} bytes (device limit {MAX_CONST_BYTES} bytes)")
        return Compiled(code, qop, flags, len(vals), bytes(blob) or b"\0\0\0\0",
                        np.asarray(offs or [0, 0], np.uint32).tobytes(), strings=vals)
    if base == "prefix":
        raise ValueError(f"column {col.name} ({col.kind}): prefix needs utf8/binary")
    rs, extra = _num_ranges(base, p.value, col, dt)
    if len(rs) > MAX_RANGES:
        raise ValueError(f"column {col.name}: {len(rs)} disjoint ranges (limit {MAX_RANGES})")
    if dt == "d16":
        # 128-bit bounds, (lo, hi) pairs of little-endian two's complement
        blob = b"".join(int(x).to_bytes(16, "little", signed=True) for r in rs for x in r)
        return Compiled(code, QOP_RANGES, flags | extra, len(rs), blob or b"\0" * 32,
                        ranges=np.array(rs, dtype=object).reshape(-1, 2))
    isf = dt in ("f4", "f8")
    cdt = np.float64 if isf else (np.uint64 if dt == "u8" else np.int64)
    arr = np.asarray(rs, dtype=cdt).reshape(-1, 2)
    return Compiled(code, QOP_RANGES, flags | extra, len(rs),
                    arr.tobytes() if len(rs) else b"\0" * 16, ranges=arr)


def compile_pred(p: Pred, col: Column, dictionary=None) -> Compiled:
    """Kernel operands of ``p`` on ``col``.  A dictionary-encoded column
    needs ``dictionary`` = (values, valid) as arrow_ipc.dictionary_values
    returns them: the predicate is evaluated on it here and becomes a
    lookup table over the indices."""
    if not col.supported:
        raise NotImplementedError(f"column {col.name}: {col.kind} columns are not scanned")
    if col.dictionary is not None:
        code = COL_CODE[col.storage]
        if p.op in ("is_null", "is_valid"):
            return Compiled(code, QOP_VALID, FLAG_NEGATE if p.op == "is_null" else 0)
        if dictionary is None:
            raise ValueError(f"column {col.name}: dictionary values needed")
        vals, dvalid = dictionary
        vcol = Column(col.name, col.kind, col.bit_width, col.signed, unit=col.unit, tz=col.tz,
                      large=col.large, precision=col.precision, scale=col.scale)
        inner = compile_pred(p, vcol)
        n = len(vals[0]) - 1 if isinstance(vals, tuple) else len(vals)
        hit = evaluate(inner, vals, dvalid, n)
        if n > MAX_LUT_BITS:
            raise ValueError(f"column {col.name}: dictionary of {n} entries (limit {MAX_LUT_BITS})")
        words = np.packbits(np.concatenate([hit, np.zeros(-n % 32 or 0, bool)]),
                            bitorder="little").view("<u4") if n else np.zeros(1, "<u4")
        return Compiled(code, QOP_LUT, 0, n, words.tobytes(), lut=hit)
    if col.kind in ("utf8", "binary"):
        code = COL_STR64 if col.large else COL_STR32
        dt = col.storage
    else:
        dt = col.storage
        if dt not in COL_CODE:
            raise NotImplementedError(f"column {col.name}: storage {dt}")
        code = COL_CODE[dt]
    return _compile_value(p, col, dt, code)


# ------------------------------------------------------------ numpy twin
def evaluate(c: Compiled, values, valid: Optional[np.ndarray], n: int) -> np.ndarray:
    """The kernel's bits for n rows on the host: values as
    arrow_ipc.decode_values returns them (indices for a LUT)."""
    ok = np.ones(n, bool) if valid is None else np.asarray(valid[:n], bool)
    if c.op == QOP_VALID:
        return ~ok if c.flags & FLAG_NEGATE else ok
    if c.op == QOP_RANGES and c.type == COL_CODE["d16"]:
        rs = [(int(a), int(b)) for a, b in c.ranges]
        hit = np.array([any(a <= int(x) <= b for a, b in rs) for x in values[:n]], bool)
        if c.flags & FLAG_NEGATE:
            hit = ~hit
        return hit & ok
    if c.op == QOP_RANGES:
        x = np.asarray(values[:n])
        if x.dtype == bool:
            x = x.astype(np.int64)
        r = c.ranges
        if x.dtype.kind == "f":
            x = x.astype(np.float64)
        elif x.dtype == np.uint64:
            pass
        else:
            x = x.astype(np.int64)
        if len(r):
            r = r.astype(x.dtype) if x.dtype.kind != "f" else r
            k = np.searchsorted(r[:, 1], x, side="left")
            kk = np.minimum(k, len(r) - 1)
            hit = (k < len(r)) & (r[kk, 0] <= x)
        else:
            hit = np.zeros(n, bool)
        if c.flags & FLAG_NAN:
            hit |= np.isnan(x)
    elif c.op in (QOP_STR_IN, QOP_STR_PREFIX):
        offs, data = values
        offs = np.asarray(offs[:n + 1], np.int64)
        ln = offs[1:] - offs[:-1]
        hit = np.zeros(n, bool)
        for s in c.strings:
            L = len(s)
            cand = np.flatnonzero(ln == L if c.op == QOP_STR_IN else ln >= L)
            if L == 0 or not len(cand):
                hit[cand] = True
                continue
            ref = np.frombuffer(s, np.uint8)
            m = data[offs[cand][:, None] + np.arange(L)[None, :]] == ref[None, :]
            hit[cand[m.all(axis=1)]] = True
    elif c.op == QOP_STR_RANGES:
        offs, data = values
        offs = np.asarray(offs[:n + 1], np.int64)
        raw = data.tobytes() if hasattr(data, "tobytes") else bytes(data)
        col = [raw[offs[i]:offs[i + 1]] for i in range(n)]
        hit = np.zeros(n, bool)
        for lo, lm, hi, hm in c.strings:
            ok_lo = [True] * n if not lm else [x >= lo if lm == 1 else x > lo for x in col]
            ok_hi = [True] * n if not hm else [x <= hi if hm == 1 else x < hi for x in col]
            hit |= np.asarray(ok_lo, bool) & np.asarray(ok_hi, bool)
    elif c.op == QOP_LUT:
        idx = np.asarray(values[:n]).astype(np.int64)
        inr = (idx >= 0) & (idx < len(c.lut))
        hit = np.zeros(n, bool)
        hit[inr] = c.lut[idx[inr]]
    else:
        raise ValueError(f"op {c.op}")
    if c.flags & FLAG_NEGATE:
        hit = ~hit
    return hit & ok


# ------------------------------------------------------------ device launch
class ColQual(C.Structure):
    """struct strom_col_qual (strom.h)."""
    _fields_ = [("type", C.c_int32), ("op", C.c_int32), ("flags", C.c_uint32),
                ("nconst", C.c_uint32), ("consts", C.c_uint64), ("offs", C.c_uint64),
                ("const_bytes", C.c_uint64), ("offs_bytes", C.c_uint64)]


# struct strom_qual_batch: values, valid, nrows, word_base, row_base, aux, aux_len
QUAL_BATCH_FIELDS = 7


def device_qual(c: Compiled, device) -> ColQual:
    """The kernel argument of ``c`` with its constants uploaded to
    ``device`` once (kept on ``c``)."""
    import torch
    key = str(device)
    if key not in c._dev:
        cs = torch.frombuffer(bytearray(c.consts or b"\0" * 4), dtype=torch.uint8).to(device)
        of = torch.frombuffer(bytearray(c.offs or b"\0" * 8), dtype=torch.uint8).to(device)
        q = ColQual(c.type, c.op, c.flags, c.nconst, cs.data_ptr(), of.data_ptr(),
                    len(c.consts), len(c.offs))
        c._dev[key] = (q, cs, of)
    return c._dev[key][0]


def qual_batched(c: Compiled, batches, nwords: int, bitmap, count, stream=None,
                 or_src=None, and_dst: bool = False) -> None:
    """One launch of the qualifier kernel over a (nbatches, 7) int64 batch
    table on the device.  bitmap[w] = (pred | or_src[w]) & (and_dst ?
    bitmap[w] : ~0); ``count`` (int64[1]) += popcount of what is written."""
    from ._util import check, lib, ptr, require_cuda, stream_handle
    require_cuda(batches, "batches")
    if batches.dim() != 2 or batches.shape[1] != QUAL_BATCH_FIELDS:
        raise ValueError("batches: int64 (n, 7)")
    if bitmap.numel() < nwords:
        raise ValueError("bitmap too small")
    q = device_qual(c, batches.device)
    check(lib().strom_column_qual(C.byref(q), ptr(batches), batches.shape[0], nwords, ptr(bitmap),
                                  ptr(or_src) if or_src is not None else 0, int(and_dst),
                                  ptr(count), stream_handle(stream)), "column_qual")
