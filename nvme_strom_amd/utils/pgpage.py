"""PostgreSQL heap-page images: builder (synthetic tables) + host reference scan.

Layout follows PostgreSQL's bufpage.h / htup_details.h (page header 24 B,
ItemIdData {lp_off:15, lp_flags:2, lp_len:15}, HeapTupleHeaderData 23 B +
null bitmap, MAXALIGN 8).  No PostgreSQL server is installed here, so these
images are the test fixtures for the GPU heap scanner and for the
SSD2RAM/SSD2GPU scan pipelines (the reference's pgsql/ extension consumes
the same page format: pgsql/nvme_strom.c:1054-1092).  Checksums use
pg_checksum_page's algorithm (host implementation in libstrom); parity with
a live PostgreSQL is unpinned.
"""
from __future__ import annotations

import struct
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .. import _native as N

SIZE_OF_PAGE_HEADER = 24
HEAP_HASNULL = 0x0001
HEAP_XMAX_LOCK_ONLY = 0x0080
HEAP_XMIN_COMMITTED = 0x0100
HEAP_XMIN_INVALID = 0x0200
HEAP_XMAX_INVALID = 0x0800
HEAP_XMIN_FROZEN = HEAP_XMIN_COMMITTED | HEAP_XMIN_INVALID   # VACUUM FREEZE / COPY FREEZE
PD_ALL_VISIBLE = 0x0004
LP_UNUSED, LP_NORMAL, LP_REDIRECT, LP_DEAD = 0, 1, 2, 3
VISIBLE = HEAP_XMIN_COMMITTED | HEAP_XMAX_INVALID


def maxalign(n: int) -> int:
    return (n + 7) & ~7


def tuple_bytes(payload: bytes, infomask: int = VISIBLE, natts: int = 1, xmin: int = 2,
                xmax: int = 0) -> bytes:
    hoff = maxalign(23)
    hdr = struct.pack("<IIIHHHHHB", xmin, xmax, 0, 0, 0, 0, natts & 0x7FF, infomask, hoff)
    assert len(hdr) == 23
    return hdr + b"\0" * (hoff - 23) + payload


def checksum(page: bytes, blkno: int) -> int:
    arr = np.frombuffer(page, dtype=np.uint8)
    return int(N.lib().strom_pg_checksum_host(arr.ctypes.data, blkno, len(page)))


def build_page(tuples: Sequence[bytes], blkno: int = 0, page_sz: int = 8192,
               with_checksum: bool = True, lp_flags: Optional[Sequence[int]] = None,
               all_visible: bool = False) -> bytes:
    """Heap page with the given tuples (each a full tuple incl. header).
    ``all_visible`` sets PD_ALL_VISIBLE in pd_flags (every tuple visible to
    every snapshot, hint bits or not)."""
    page = bytearray(page_sz)
    upper = page_sz
    lps = []
    for i, t in enumerate(tuples):
        upper = (upper - len(t)) & ~7
        page[upper:upper + len(t)] = t
        flags = LP_NORMAL if lp_flags is None else lp_flags[i]
        lps.append(upper | (flags << 15) | (len(t) << 17))
    lower = SIZE_OF_PAGE_HEADER + 4 * len(lps)
    if lower > upper:
        raise ValueError("tuples do not fit")
    for i, lp in enumerate(lps):
        struct.pack_into("<I", page, SIZE_OF_PAGE_HEADER + 4 * i, lp)
    # pd_lsn, pd_checksum, pd_flags, pd_lower, pd_upper, pd_special, pd_psv, pd_prune_xid
    flags = PD_ALL_VISIBLE if all_visible else 0
    struct.pack_into("<QHHHHHHI", page, 0, 1, 0, flags, lower, upper, page_sz, page_sz | 4, 0)
    if with_checksum:
        struct.pack_into("<H", page, 8, checksum(bytes(page), blkno))
    return bytes(page)


def int_tuples(values: Iterable[int], width: int = 8, invisible: Iterable[int] = (),
               pad: int = 0, frozen: Iterable[int] = (), nohint: Iterable[int] = ()) -> List[bytes]:
    """One fixed-width int column (+ ``pad`` filler bytes) per tuple.

    Row i carries: xmin aborted (``invisible``), xmin frozen + xmax invalid
    (``frozen``), no hint bits at all (``nohint``: visible only on an
    all-visible page), else xmin committed + xmax invalid."""
    inv, frz, noh = set(invisible), set(frozen), set(nohint)
    fmt = "<q" if width == 8 else "<i"
    out = []
    for i, v in enumerate(values):
        if i in inv:
            mask = HEAP_XMIN_INVALID | HEAP_XMAX_INVALID
        elif i in frz:
            mask = HEAP_XMIN_FROZEN | HEAP_XMAX_INVALID
        elif i in noh:
            mask = 0
        else:
            mask = VISIBLE
        out.append(tuple_bytes(struct.pack(fmt, v) + b"\xAB" * pad, infomask=mask))
    return out


def build_table(values: np.ndarray, per_page: int, width: int = 8, page_sz: int = 8192,
                with_checksum: bool = True, invisible_every: int = 0,
                blkno_base: int = 0, frozen_every: int = 0,
                all_visible_every: int = 0) -> bytes:
    """A relation of pages, ``per_page`` int tuples each.

    ``frozen_every``: every k-th row is frozen (both xmin hint bits).
    ``all_visible_every``: every k-th page has PD_ALL_VISIBLE set and its
    rows carry no hint bits (VACUUM set the flag, nobody hinted the rows)."""
    pages = []
    for p, i0 in enumerate(range(0, len(values), per_page)):
        chunk = values[i0:i0 + per_page]
        allvis = bool(all_visible_every) and p % all_visible_every == 0
        rows = range(len(chunk))
        if allvis:
            inv, frz, noh = [], [], list(rows)
        else:
            inv = [j for j in rows if invisible_every and (i0 + j) % invisible_every == 0]
            frz = [j for j in rows if frozen_every and (i0 + j) % frozen_every == 1 % frozen_every
                   and j not in inv]
            noh = []
        pages.append(build_page(int_tuples(chunk.tolist(), width, inv, frozen=frz, nohint=noh),
                                blkno_base + p, page_sz, with_checksum, all_visible=allvis))
    return b"".join(pages)


def tuple_visible(infomask: int, pd_flags: int) -> bool:
    """Hint-bit visibility as the GPU scanner applies it (no clog access):
    every tuple of a PD_ALL_VISIBLE page is visible (reference
    pgsql/nvme_strom.c:870-891 sends such pages to DMA unchecked); else
    xmin must be known committed (HEAP_XMIN_COMMITTED, which a frozen xmin
    also carries) and xmax invalid or lock-only."""
    if pd_flags & PD_ALL_VISIBLE:
        return True
    if not infomask & HEAP_XMIN_COMMITTED:
        return False
    return bool(infomask & (HEAP_XMAX_INVALID | HEAP_XMAX_LOCK_ONLY))


def host_scan(data: bytes, page_sz: int = 8192, skip_invisible: bool = False,
              attr_off: int = -1, attr_width: int = 8, lo: int = -(1 << 63),
              hi: int = (1 << 63) - 1, verify_checksum: bool = False,
              blkno_base: int = 0) -> Tuple[List[int], List[int]]:
    """Reference scan: (sorted item ids page<<16|lineno, per-page status)."""
    items, status = [], []
    for pg in range(len(data) // page_sz):
        page = data[pg * page_sz:(pg + 1) * page_sz]
        ck, flags, lower, upper, special, psv = struct.unpack_from("<HHHHHH", page, 8)
        st = 0
        if upper == 0:
            st |= 4
        elif (lower < 24 or lower > upper or upper > special or special > page_sz or special & 7
              or flags & ~7 or (psv & 0xFF00) != (page_sz & 0xFF00)):
            st |= 1
        if verify_checksum and not st:
            if checksum(page, blkno_base + pg) != ck:
                st |= 2
        status.append(st)
        if st:
            continue
        for i in range((lower - 24) // 4):
            lp, = struct.unpack_from("<I", page, 24 + 4 * i)
            off, fl, ln = lp & 0x7FFF, (lp >> 15) & 3, lp >> 17
            if fl != LP_NORMAL or ln < 23 or off < 24 or off + ln > page_sz:
                continue
            infomask, = struct.unpack_from("<H", page, off + 20)
            hoff = page[off + 22]
            if skip_invisible and not tuple_visible(infomask, flags):
                continue
            if attr_off >= 0:
                at = hoff + attr_off
                if infomask & HEAP_HASNULL or at + attr_width > ln:
                    continue
                v, = struct.unpack_from("<q" if attr_width == 8 else "<i", page, off + at)
                if not (lo <= v <= hi):
                    continue
            items.append((pg << 16) | (i + 1))
    return sorted(items), status
