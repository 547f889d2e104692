"""PostgreSQL heap-page scan on the GPU (csrc/kernels/heapscan.hip)."""
from __future__ import annotations

import ctypes as C
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

    def sorted_items(self) -> np.ndarray:
        return np.sort(self.items[:self.count].cpu().numpy().view(np.uint32))


def heap_scan(pages: torch.Tensor, page_sz: int = 8192, verify_checksum: bool = False,
              skip_invisible: bool = False, attr_off: int = -1, attr_width: int = 4,
              lo: int = -(1 << 63), hi: int = (1 << 63) - 1, blkno_base: int = 0,
              out_cap: Optional[int] = None, blknos: Optional[torch.Tensor] = None,
              stream=None) -> HeapScanResult:
    """Scan ``pages`` (uint8, npages*page_sz) for visible LP_NORMAL tuples,
    optionally filtered by lo <= int column at ``attr_off`` (after t_hoff) <= hi."""
    require_cuda(pages, "pages")
    pages = pages.view(torch.uint8)
    if pages.numel() % page_sz:
        raise ValueError("pages is not a whole number of pages")
    npages = pages.numel() // page_sz
    cap = out_cap if out_cap is not None else npages * (page_sz // 28 + 1)
    items = torch.empty(max(cap, 1), dtype=torch.int32, device=pages.device)
    count = torch.zeros(1, dtype=torch.int32, device=pages.device)
    status = torch.empty(max(npages, 1), dtype=torch.int32, device=pages.device)
    flags = (VERIFY_CHECKSUM if verify_checksum else 0) | (SKIP_INVISIBLE if skip_invisible else 0)
    a = N.HeapScanArgs(pages=ptr(pages), npages=npages, page_sz=page_sz, flags=flags,
                       attr_off=attr_off, attr_width=attr_width, lo=lo, hi=hi,
                       out_items=ptr(items), out_cap=cap, out_count=ptr(count),
                       page_status=ptr(status), blkno_base=blkno_base,
                       blknos=ptr(blknos) if blknos is not None else None)
    check(lib().strom_heap_scan(C.byref(a), stream_handle(stream)), "heap_scan")
    n = int(count.item())
    return HeapScanResult(items, min(n, cap), status[:npages])


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
    """ctypes strom_heap_qual list (sorted by attribute) of pgtuple.Qual."""
    import struct
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
                s.lo, s.hi = int(args[0]), int(args[1])
            else:
                raise ValueError(f"range qual on a {desc.types[k]} column")
        elif op == "in":
            vals = [int(v) for v in args[0]]
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


@dataclass
class HeapScan2Result(HeapScanResult):
    recheck: int = 0                     # undecidable tuples (pages flagged PAGE_RECHECK)


def heap_scan2(pages: torch.Tensor, desc, quals, page_sz: int = 8192,
               verify_checksum: bool = False, skip_invisible: bool = False,
               blkno_base: int = 0, out_cap: Optional[int] = None,
               blknos: Optional[torch.Tensor] = None, stream=None,
               sync: bool = True) -> HeapScan2Result:
    """Scan ``pages`` deforming every tuple with ``desc`` (utils.pgtuple) and
    keeping the ones that pass every qualifier of ``quals`` (ANDed).
    ``sync=False`` leaves ``count`` / ``recheck`` as device tensors (no host
    read)."""
    require_cuda(pages, "pages")
    pages = pages.view(torch.uint8)
    if pages.numel() % page_sz:
        raise ValueError("pages is not a whole number of pages")
    npages = pages.numel() // page_sz
    cap = out_cap if out_cap is not None else npages * (page_sz // 28 + 1)
    dev = pages.device
    items = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    cnt = torch.zeros(2, dtype=torch.int32, device=dev)      # [count, recheck]
    status = torch.empty(max(npages, 1), dtype=torch.int32, device=dev)
    flags = (VERIFY_CHECKSUM if verify_checksum else 0) | (SKIP_INVISIBLE if skip_invisible else 0)
    g = N.HeapScan2Args()
    g.base = N.HeapScanArgs(pages=ptr(pages), npages=npages, page_sz=page_sz, flags=flags,
                            attr_off=-1, attr_width=8, lo=0, hi=0,
                            out_items=ptr(items), out_cap=cap, out_count=ptr(cnt),
                            page_status=ptr(status), blkno_base=blkno_base,
                            blknos=ptr(blknos) if blknos is not None else None)
    g.desc = tupdesc_struct(desc)
    qs = qual_structs(desc, quals)
    g.nquals = len(qs)
    for i, q in enumerate(qs):
        g.quals[i] = q
    g.recheck_count = ptr(cnt) + 4
    if npages:
        cnt[1].zero_()
    check(lib().strom_heap_scan2(C.byref(g), stream_handle(stream)), "heap_scan2")
    if not sync:
        r = HeapScan2Result(items, cnt[0:1], status[:npages])
        r.recheck = cnt[1:2]
        return r
    c = cnt.cpu().tolist()
    r = HeapScan2Result(items, min(c[0], cap), status[:npages])
    r.recheck = c[1]
    return r


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
