"""PostgreSQL heap-page scan on the GPU (csrc/kernels/heapscan.hip)."""
from __future__ import annotations

import ctypes as C
import math
import struct
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .. import _native as N
from ._util import check, lib, ptr, require_cuda, stream_handle

VERIFY_CHECKSUM = 1
SKIP_INVISIBLE = 2
PAGE_BAD_HEADER = 1
PAGE_BAD_CHECKSUM = 2
PAGE_EMPTY = 4


@dataclass
class HeapScanResult:
    items: torch.Tensor        # int32 (page << 16 | lineno), unordered
    count: int
    page_status: torch.Tensor  # int32 per page (PAGE_* bits)
    # snapshot mode (mvcc=): tuples the device check removed; tuples it could
    # not decide (kept, their pages flagged PAGE_RECHECK) add to ``recheck``
    removed: int = 0
    recheck: int = 0

    def sorted_items(self) -> np.ndarray:
        return np.sort(self.items[:self.count].cpu().numpy().view(np.uint32))


class DeviceMvcc:
    """HeapTupleSatisfiesMVCC's inputs in HBM for the scan kernels' snapshot
    check: the snapshot (xip / subxip / the scanning transaction's xids,
    sorted for the device's binary search), and the pg_xact, pg_subtrans and
    pg_multixact windows (utils.pgmvcc objects).  Uploaded once — a scan
    builds one per run and every chunk's launch reads it — and kept alive by
    this object; ``struct`` is the strom_pg_mvcc of device pointers, plus
    the running-xid bitmap over [xmin, xmax) (``running``)."""

    RUNNING_MAX_BITS = 1 << 23

    def __init__(self, snap, clog=None, subtrans=None, multi=None, device="cuda"):
        dev = torch.device(device)
        self.device = dev
        self._keep = []
        m = N.PgMvcc()

        def up(a: np.ndarray):
            a = np.ascontiguousarray(a)
            if a.size == 0:
                return None
            t = torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(dev)
            self._keep.append(t)
            return ptr(t)

        def xids(v):
            return np.unique(np.asarray([int(x) & 0xFFFFFFFF for x in v], dtype=np.uint32))
        m.xmin, m.xmax = snap.xmin & 0xFFFFFFFF, snap.xmax & 0xFFFFFFFF
        xip, sub, cur = xids(snap.xip), xids(snap.subxip), xids(snap.curxids)
        m.xip, m.nxip = up(xip), len(xip)
        m.subxip, m.nsubxip = up(sub), len(sub)
        m.curxids, m.ncurxids = up(cur), len(cur)
        m.suboverflowed = int(bool(snap.suboverflowed))
        m.curcid = snap.curcid
        if clog is not None:
            m.clog, m.clog_n, m.clog_base = up(clog.bits), clog.nxids, clog.base
        if subtrans is not None:
            m.subtrans, m.subtrans_n = up(subtrans.parent), len(subtrans.parent)
            m.subtrans_base = subtrans.base
        if multi is not None:
            off, mem = multi.offsets_array(), multi.members_pages()
            m.mx_offsets, m.mx_base, m.mx_n = up(off), multi.base, len(off) - 1
            m.mx_members, m.mxm_n, m.mxm_base = up(mem), len(multi.members), multi.members_base
        # XidInMVCCSnapshot's list searches as one bit test: xip (and subxip
        # unless the snapshot overflowed) over [xmin, xmax), up to 2^23 xids
        span = (m.xmax - m.xmin) & 0xFFFFFFFF
        self.running, self.running_bits = None, 0
        if 0 < span <= self.RUNNING_MAX_BITS:
            bm = np.zeros((span + 31) // 32, dtype=np.uint32)
            members = [xip] if snap.suboverflowed else [xip, sub]
            for arr in members:
                k = (arr.astype(np.int64) - m.xmin) & 0xFFFFFFFF
                k = k[k < span]
                np.bitwise_or.at(bm, k >> 5, (np.uint32(1) << (k & 31).astype(np.uint32)))
            self._run_t = torch.from_numpy(bm.view(np.uint8).copy()).to(dev)
            self.running, self.running_bits = ptr(self._run_t), span
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()
        self.struct = m


def _mvcc_pages(mvcc_pages, npages: int, dev):
    """The per-page check flags as a device uint8 tensor (None: every page
    that is not PD_ALL_VISIBLE is checked)."""
    if mvcc_pages is None:
        return None
    t = mvcc_pages if isinstance(mvcc_pages, torch.Tensor) else torch.from_numpy(
        np.ascontiguousarray(np.asarray(mvcc_pages, dtype=np.uint8)))
    t = t.to(device=dev, dtype=torch.uint8)
    if t.numel() < npages:
        raise ValueError(f"mvcc_pages has {t.numel()} entries for {npages} pages")
    return t


def heap_scan(pages: torch.Tensor, page_sz: int = 8192, verify_checksum: bool = False,
              skip_invisible: bool = False, attr_off: int = -1, attr_width: int = 4,
              lo: int = -(1 << 63), hi: int = (1 << 63) - 1, blkno_base: int = 0,
              out_cap: Optional[int] = None, blknos: Optional[torch.Tensor] = None,
              stream=None, mvcc: Optional[DeviceMvcc] = None, mvcc_pages=None) -> HeapScanResult:
    """Scan ``pages`` (uint8, npages*page_sz) for visible LP_NORMAL tuples,
    optionally filtered by lo <= int column at ``attr_off`` (after t_hoff) <= hi.
    ``mvcc`` (a DeviceMvcc): every tuple of a page that is not PD_ALL_VISIBLE
    (and whose ``mvcc_pages`` flag, when given, is nonzero) is checked
    against the snapshot on the device."""
    require_cuda(pages, "pages")
    pages = pages.view(torch.uint8)
    if pages.numel() % page_sz:
        raise ValueError("pages is not a whole number of pages")
    npages = pages.numel() // page_sz
    cap = out_cap if out_cap is not None else npages * (page_sz // 28 + 1)
    items = torch.empty(max(cap, 1), dtype=torch.int32, device=pages.device)
    cnt = torch.zeros(3, dtype=torch.int32, device=pages.device)   # count, recheck, removed
    status = torch.empty(max(npages, 1), dtype=torch.int32, device=pages.device)
    flags = (VERIFY_CHECKSUM if verify_checksum else 0) | (SKIP_INVISIBLE if skip_invisible else 0)
    a = N.HeapScanArgs(pages=ptr(pages), npages=npages, page_sz=page_sz, flags=flags,
                       attr_off=attr_off, attr_width=attr_width, lo=lo, hi=hi,
                       out_items=ptr(items), out_cap=cap, out_count=ptr(cnt),
                       page_status=ptr(status), blkno_base=blkno_base,
                       blknos=ptr(blknos) if blknos is not None else None)
    if mvcc is None:
        check(lib().strom_heap_scan(C.byref(a), stream_handle(stream)), "heap_scan")
    else:
        mp = _mvcc_pages(mvcc_pages, npages, pages.device)
        check(lib().strom_heap_scan_mvcc(C.byref(a), C.byref(mvcc.struct),
                                         ptr(mp) if mp is not None else None, ptr(cnt) + 8,
                                         ptr(cnt) + 4, mvcc.running, mvcc.running_bits,
                                         stream_handle(stream)), "heap_scan_mvcc")
    c = cnt.cpu().tolist()
    return HeapScanResult(items, min(c[0], cap), status[:npages], removed=c[2], recheck=c[1])


# ------------------------------------------------- tuple descriptor + quals
PAGE_RECHECK = 8
QUAL_KIND = {"between": 1, "isnull": 3, "notnull": 4, "text_eq": 5, "prefix": 6, "in": 7}


def tupdesc_struct(desc) -> N.HeapTupDesc:
    """ctypes strom_heap_tupdesc of a utils.pgtuple.TupleDesc."""
    if not 1 <= desc.natts <= N.HEAP_MAX_ATTS:
        raise ValueError(f"{desc.natts} attributes (1..{N.HEAP_MAX_ATTS})")
    d = N.HeapTupDesc()
    d.natts = desc.natts
    for i, (L, al, co) in enumerate(zip(desc.attlen, desc.attalign, desc.cacheoff())):
        d.attlen[i], d.attalign[i], d.cacheoff[i] = L, al, co
    return d


def qual_structs(desc, quals) -> list:
    """ctypes strom_heap_qual list (sorted by attribute) of pgtuple.Qual:
    the fixed-size form (<= 8 ANDed quals, <= 32 constant bytes); heap_scan2
    compiles a Program instead."""
    import math
    out = []
    for q in quals:
        k = desc.attno(q.col)
        kind = desc.kinds[k]
        s = N.HeapQual()
        s.attno = k
        op = q.op
        if op == "eq":
            op, args = "between", (q.args[0], q.args[0])
        else:
            args = q.args
        if op == "between":
            if kind == "float":
                s.kind = 2
                s.lo = struct.unpack("<q", struct.pack("<d", float(args[0])))[0]
                s.hi = struct.unpack("<q", struct.pack("<d", float(args[1])))[0]
            elif kind == "int":
                s.kind = 1
                # exact: a fractional lower bound rounds up, an upper one
                # down; non-finite bounds clamp (an empty range: lo > hi)
                b = _int_bounds("between", args, -(1 << 63), (1 << 63) - 1)
                s.lo, s.hi = b if b is not None else (1, 0)
            else:
                raise ValueError(f"range qual on a {desc.types[k]} column")
        elif op == "in":
            vals = [int(v) for v in args[0] if _is_int_value(v)]
            if kind != "int" or len(vals) > 4:
                raise ValueError("IN lists take up to 4 values of an int column")
            s.kind, s.nconst = 7, len(vals)
            raw = struct.pack(f"<{len(vals)}q", *vals)
            C.memmove(C.addressof(s.cbytes), raw, len(raw))
        elif op in ("text_eq", "prefix"):
            c = args[0].encode() if isinstance(args[0], str) else bytes(args[0])
            if desc.attlen[k] != -1 or len(c) > 32:
                raise ValueError("text quals take a varlena column and <= 32 bytes")
            s.kind, s.nconst = QUAL_KIND[op], len(c)
            C.memmove(C.addressof(s.cbytes), c, len(c))
        else:
            s.kind = QUAL_KIND[op]
        out.append(s)
    out.sort(key=lambda s: s.attno)
    if len(out) > N.HEAP_MAX_QUALS:
        raise ValueError(f"more than {N.HEAP_MAX_QUALS} quals")
    return out


QUAL_TEXT_IN, QUAL_NUMERIC_RANGE = 8, 9
QUAL2_FALSE = 0x80
_INT_LIMITS = {1: (-(1 << 7), (1 << 7) - 1), 2: (-(1 << 15), (1 << 15) - 1),
               4: (-(1 << 31), (1 << 31) - 1), 8: (-(1 << 63), (1 << 63) - 1)}


class Program:
    """A qualifier list compiled for strom_heap_scan2's program mode: one
    strom_heap_qual2 per leaf qualifier, clause ids for the CNF (a ``Qual``
    is a clause of its own, an ``Or`` one clause of several), and the
    constant pool (IN lists and text of any size, numeric constants)."""

    def __init__(self, desc, quals):
        import math
        from ..utils import pgtuple as T
        self.pool = bytearray()
        self.quals: list = []

        def const(b: bytes) -> int:
            while len(self.pool) % 8:
                self.pool.append(0)
            o = len(self.pool)
            self.pool += b
            return o

        def num_const(v) -> int:
            kind, neg, weight, digits, _ = T.numeric_parts(v)
            return const(struct.pack("<HHhH", kind, neg, weight, len(digits)) +
                         struct.pack(f"<{len(digits)}h", *digits))

        def emit(k, kind, clause, nconst=0, coff=0, lo=0, hi=0, flags=0):
            q = N.HeapQual2()
            q.attno, q.kind, q.flags, q.clause = k, kind, flags, clause
            q.nconst, q.coff, q.lo, q.hi = nconst, coff, lo, hi
            self.quals.append(q)

        def never(k, clause):
            # a constant-false qual (false for NULLs and unreadable values too)
            emit(k, 4, clause, flags=QUAL2_FALSE)

        for ci, clause in enumerate(T.clauses(quals)):
            for q in clause:
                k = desc.attno(q.col)
                kind, L = desc.kinds[k], desc.attlen[k]
                op, args = q.op, q.args
                if op == "isnull":
                    emit(k, 3, ci)
                elif op == "notnull":
                    emit(k, 4, ci)
                elif op in ("text_eq", "prefix", "text_in"):
                    if L != -1 or kind not in ("text",):
                        raise ValueError(f"{op} on a {desc.types[k]} column")
                    if op == "text_in":
                        vals = [T._b(c) for c in args[0]]
                        offs = [const(v) for v in vals]
                        table = b"".join(struct.pack("<II", o, len(v)) for o, v in zip(offs, vals))
                        emit(k, QUAL_TEXT_IN, ci, nconst=len(vals), coff=const(table))
                    else:
                        c = T._b(args[0])
                        emit(k, 5 if op == "text_eq" else 6, ci, nconst=len(c), coff=const(c))
                elif kind == "numeric":
                    if op == "in":
                        for c in args[0]:
                            o = num_const(c)
                            emit(k, QUAL_NUMERIC_RANGE, ci, lo=o, hi=o)
                        if not args[0]:
                            never(k, ci)
                        continue
                    lo = hi = None
                    flags = 0
                    if op == "between":
                        lo, hi = args
                    elif op == "eq":
                        lo = hi = args[0]
                    elif op in ("lt", "le"):
                        hi = args[0]
                        flags |= 1 | (8 if op == "lt" else 0)
                    elif op in ("gt", "ge"):
                        lo = args[0]
                        flags |= 2 | (4 if op == "gt" else 0)
                    else:
                        raise ValueError(f"{op} on a numeric column")
                    emit(k, QUAL_NUMERIC_RANGE, ci, flags=flags,
                         lo=num_const(lo) if lo is not None else 0,
                         hi=num_const(hi) if hi is not None else 0)
                elif kind == "float":
                    if op == "in":
                        for c in args[0]:
                            emit(k, 2, ci, lo=_fbits(c), hi=_fbits(c))
                        if not args[0]:
                            never(k, ci)
                        continue
                    lo, hi = -math.inf, math.inf
                    if op == "between":
                        lo, hi = float(args[0]), float(args[1])
                    elif op == "eq":
                        lo = hi = float(args[0])
                    elif op == "le":
                        hi = float(args[0])
                    elif op == "lt":
                        hi = math.nextafter(float(args[0]), -math.inf)
                    elif op == "ge":
                        lo = float(args[0])
                    elif op == "gt":
                        lo = math.nextafter(float(args[0]), math.inf)
                    else:
                        raise ValueError(f"{op} on a float column")
                    emit(k, 2, ci, lo=_fbits(lo), hi=_fbits(hi))
                elif kind == "int" and L in _INT_LIMITS:
                    tmin, tmax = _INT_LIMITS[L]
                    if op == "in":
                        vals = sorted({int(c) for c in args[0] if _is_int_value(c)
                                       and tmin <= int(c) <= tmax})
                        if not vals:
                            never(k, ci)
                            continue
                        emit(k, 7, ci, nconst=len(vals),
                             coff=const(struct.pack(f"<{len(vals)}q", *vals)))
                        continue
                    b = _int_bounds(op, args, tmin, tmax)
                    if b is None:
                        never(k, ci)
                    else:
                        emit(k, 1, ci, lo=b[0], hi=b[1])
                else:
                    raise ValueError(f"{op} on a {desc.types[k]} column")
        # clauses by their first attribute, quals by attribute inside a
        # clause: the device deforms each tuple forward, walking again from
        # the start only when a clause goes back to an earlier attribute
        groups: dict = {}
        for q in self.quals:
            groups.setdefault(q.clause, []).append(q)
        order = sorted(groups.values(), key=lambda g: min(q.attno for q in g))
        self.quals = []
        for ci, g in enumerate(order):
            for q in sorted(g, key=lambda q: q.attno):
                q.clause = ci
                self.quals.append(q)
        # the device reads the pool a dword at a time: padded to 8 bytes
        while not self.pool or len(self.pool) % 8:
            self.pool.append(0)
        self._dev: dict = {}
        self._checked: set = set()        # tuple descriptors the program passed
        self._arrays = None

    def device_arrays(self, dev, stream) -> tuple:
        """(program, pool) as device tensors on ``dev``: uploaded once (on
        ``stream``, waited for) and reused by every later scan with this
        program — two small host-to-device copies per launch cost ~20 % of
        an in-HBM scan of 1 GiB (profiles/r5/heap/prog_kbench.md)."""
        key = (dev.type, dev.index)
        c = self._dev.get(key)
        if c is None:
            raw, pool = self.arrays()
            with torch.cuda.stream(stream):
                d_prog = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
                d_pool = torch.frombuffer(bytearray(pool), dtype=torch.uint8).to(dev)
            stream.synchronize()
            c = self._dev[key] = (d_prog, d_pool)
        return c

    def fixed(self):
        """The program as strom_heap_scan2's fixed-size AND list (the quals
        ride in the kernel arguments: scalar loads and an early exit per
        tuple), or None when it needs the program mode: an OR, more than
        HEAP_MAX_QUALS quals, a kind or constant the fixed form lacks."""
        qs = self.quals
        if len(qs) > N.HEAP_MAX_QUALS or len({q.clause for q in qs}) != len(qs):
            return None
        out = []
        for q in qs:
            if q.flags or q.kind not in (1, 2, 3, 4, 5, 6, 7):
                return None
            s = N.HeapQual()
            s.attno, s.kind, s.lo, s.hi = q.attno, q.kind, q.lo, q.hi
            if q.kind in (5, 6, 7):
                n = q.nconst * (8 if q.kind == 7 else 1)
                if q.nconst > (4 if q.kind == 7 else 32):
                    return None
                s.nconst = q.nconst
                C.memmove(C.addressof(s.cbytes), bytes(self.pool[q.coff:q.coff + n]), n)
            out.append(s)
        if any(b.attno < a.attno for a, b in zip(out, out[1:])):
            return None
        return out

    def arrays(self):
        """(program bytes, pool bytes) for upload (a program is not changed
        after compilation: built once)."""
        if self._arrays is None:
            self._arrays = (b"".join(bytes(q) for q in self.quals), bytes(self.pool))
        return self._arrays


def _is_int_value(c) -> bool:
    """A constant equal to some integer (NaN and the infinities are not)."""
    d = _exact(c)
    return d.is_finite() and d == int(d)


def _int_bounds(op: str, args, tmin: int, tmax: int):
    """Exact [lo, hi] of an int qualifier on a column of range [tmin, tmax]
    (a fractional lower bound rounds up, an upper one down; clamped to the
    type), or None when nothing qualifies.  Non-finite constants compare as
    PostgreSQL / IEEE do: -inf below and +inf above every integer, NaN
    (equal to nothing, ordered by nothing here) never true."""
    from decimal import Decimal
    d = [_exact(a) for a in args]
    if any(x.is_nan() for x in d):
        return None

    def lo_of(x: Decimal, strict: bool) -> int:
        if x.is_infinite():
            return tmin if x < 0 else tmax + 1
        return math.floor(x) + 1 if strict else math.ceil(x)

    def hi_of(x: Decimal, strict: bool) -> int:
        if x.is_infinite():
            return tmin - 1 if x < 0 else tmax
        return math.ceil(x) - 1 if strict else math.floor(x)
    lo, hi = tmin, tmax
    if op == "between":
        lo, hi = lo_of(d[0], False), hi_of(d[1], False)
    elif op == "eq":
        lo, hi = lo_of(d[0], False), hi_of(d[0], False)
    elif op == "le":
        hi = hi_of(d[0], False)
    elif op == "lt":
        hi = hi_of(d[0], True)
    elif op == "ge":
        lo = lo_of(d[0], False)
    elif op == "gt":
        lo = lo_of(d[0], True)
    else:
        raise ValueError(f"{op} on an int column")
    lo, hi = max(lo, tmin), min(hi, tmax)
    return None if lo > hi else (lo, hi)


def _exact(x):
    """The exact value of an int / float / Decimal constant (a float's binary
    value, as Python's int-vs-float comparisons use)."""
    from decimal import Decimal
    return x if isinstance(x, Decimal) else Decimal(x)


def _fbits(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", float(x)))[0]


@dataclass
class HeapScan2Result(HeapScanResult):
    pass                                 # recheck: undecidable tuples (pages flagged PAGE_RECHECK)


def heap_scan2(pages: torch.Tensor, desc, quals, page_sz: int = 8192,
               verify_checksum: bool = False, skip_invisible: bool = False,
               blkno_base: int = 0, out_cap: Optional[int] = None,
               blknos: Optional[torch.Tensor] = None, stream=None,
               sync: bool = True, program: bool = False,
               mvcc: Optional[DeviceMvcc] = None, mvcc_pages=None) -> HeapScan2Result:
    """Scan ``pages`` deforming every tuple with ``desc`` (utils.pgtuple) and
    keeping the ones ``quals`` selects: a list of ``pgtuple.Qual`` (ANDed)
    and ``pgtuple.Or`` clauses (CNF), or a compiled ``Program``.
    ``sync=False`` leaves ``count`` / ``recheck`` / ``removed`` as device
    tensors (no host read); ``program=True`` runs the program mode even for a
    plain AND list; ``mvcc`` / ``mvcc_pages``: the snapshot check, as in
    :func:`heap_scan`."""
    require_cuda(pages, "pages")
    pages = pages.view(torch.uint8)
    if pages.numel() % page_sz:
        raise ValueError("pages is not a whole number of pages")
    npages = pages.numel() // page_sz
    cap = out_cap if out_cap is not None else npages * (page_sz // 28 + 1)
    dev = pages.device
    items = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    cnt = torch.zeros(3, dtype=torch.int32, device=dev)      # [count, recheck, removed]
    status = torch.empty(max(npages, 1), dtype=torch.int32, device=dev)
    flags = (VERIFY_CHECKSUM if verify_checksum else 0) | (SKIP_INVISIBLE if skip_invisible else 0)
    g = N.HeapScan2Args()
    g.base = N.HeapScanArgs(pages=ptr(pages), npages=npages, page_sz=page_sz, flags=flags,
                            attr_off=-1, attr_width=8, lo=0, hi=0,
                            out_items=ptr(items), out_cap=cap, out_count=ptr(cnt),
                            page_status=ptr(status), blkno_base=blkno_base,
                            blknos=ptr(blknos) if blknos is not None else None)
    g.desc = tupdesc_struct(desc)
    # the qualifier list as a program (CNF, any number of quals and
    # constants) in device memory, checked on its host copy first; a plain
    # AND list of the fixed form's kinds goes in the arguments instead
    prog = quals if isinstance(quals, Program) else Program(desc, quals)
    raw, pool = prog.arrays()
    fx = prog.fixed() if prog.quals and not program else None
    keep = []
    if fx is not None:
        # a plain AND list: the fixed-size form in the kernel arguments
        g.nquals = len(fx)
        for i, q in enumerate(fx):
            g.quals[i] = q
    elif prog.quals:
        # checked once per program and tuple descriptor
        dkey = bytes(g.desc)
        if dkey not in prog._checked:
            hp = np.frombuffer(raw, np.uint8)
            check(lib().strom_heap_prog_check(C.byref(g.desc), hp.ctypes.data, len(prog.quals),
                                              pool, len(pool)), "heap_scan2 program")
            prog._checked.add(dkey)
        # uploaded once per program and device (complete before any launch
        # reads it), kept by the program and by the result
        ts = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.current_stream(dev)
        d_prog, d_pool = prog.device_arrays(dev, ts)
        g.prog, g.cpool = ptr(d_prog), ptr(d_pool)
        g.nprog, g.cpool_len = len(prog.quals), len(pool)
        keep = [d_prog, d_pool]
    g.recheck_count = ptr(cnt) + 4
    if mvcc is not None:
        mp = _mvcc_pages(mvcc_pages, npages, dev)
        g.mvcc, g.mvcc_on = mvcc.struct, 1
        g.mvcc_pages = ptr(mp) if mp is not None else None
        g.mvcc_removed = ptr(cnt) + 8
        g.mvcc_running, g.mvcc_running_bits = mvcc.running, mvcc.running_bits
        keep = keep + [mp, mvcc]
    check(lib().strom_heap_scan2(C.byref(g), stream_handle(stream)), "heap_scan2")
    if not sync:
        r = HeapScan2Result(items, cnt[0:1], status[:npages])
        r.recheck = cnt[1:2]
        r.removed = cnt[2:3]
        r.keep = keep
        return r
    c = cnt.cpu().tolist()
    return HeapScan2Result(items, min(c[0], cap), status[:npages], removed=c[2], recheck=c[1])


def heap_project(pages: torch.Tensor, items: torch.Tensor, count: torch.Tensor, desc, col,
                 page_sz: int = 8192, cap: Optional[int] = None, stream=None):
    """One attribute of the tuples ``items`` names (count: device u32/i32[1]):
    (values, valid) — values int64 (float columns: float64) of length cap,
    valid uint8 (0 NULL, 1 value, 2 compressed / out-of-line varlena).  For
    varlena columns a value is (byte offset in ``pages`` << 32 | length)."""
    require_cuda(pages, "pages")
    k = desc.attno(col)
    as_float = desc.kinds[k] == "float"
    n = int(cap if cap is not None else items.numel())
    dev = pages.device
    vals = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    valid = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    d = tupdesc_struct(desc)
    check(lib().strom_heap_project(ptr(pages), page_sz, ptr(items), ptr(count), n, C.byref(d), k,
                                   1 if as_float else 0, ptr(vals), ptr(valid),
                                   stream_handle(stream)), "heap_project")
    if as_float:
        vals = vals.view(torch.float64)
    return vals[:n], valid[:n]


def heap_project_many(pages: torch.Tensor, items: torch.Tensor, count: torch.Tensor, desc, cols,
                      page_sz: int = 8192, cap: Optional[int] = None, stream=None) -> dict:
    """Several attributes of the tuples ``items`` names, in one deform walk
    per tuple: {column: (values, valid)} as heap_project returns them."""
    require_cuda(pages, "pages")
    cols = list(cols)
    ks = [desc.attno(c) for c in cols]
    if len(set(ks)) != len(ks):
        raise ValueError("a column is projected twice")
    n = int(cap if cap is not None else items.numel())
    dev = pages.device
    m = max(n, 1)
    vals = torch.empty((len(cols), m), dtype=torch.int64, device=dev)
    valid = torch.empty((len(cols), m), dtype=torch.uint8, device=dev)
    fmask = sum(1 << j for j, k in enumerate(ks) if desc.kinds[k] == "float")
    att = (C.c_int32 * len(ks))(*ks)
    d = tupdesc_struct(desc)
    check(lib().strom_heap_project_n(ptr(pages), page_sz, ptr(items), ptr(count), n, C.byref(d),
                                     C.addressof(att), len(ks), fmask, ptr(vals), ptr(valid),
                                     stream_handle(stream)), "heap_project_n")
    out = {}
    for j, c in enumerate(cols):
        v = vals[j, :n]
        out[c] = (v.view(torch.float64) if (fmask >> j) & 1 else v, valid[j, :n])
    return out
