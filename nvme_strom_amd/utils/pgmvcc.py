"""PostgreSQL MVCC inputs for the heap scan: the visibility-map fork, a
commit log and snapshots.

The reference routes each block of a chunk by the visibility map: blocks
that are all-visible (and not in shared buffers) go to NVMe DMA unchecked,
the rest are read through the buffer manager and every tuple is checked
against the scan's snapshot, invisible ones marked unused
(pgsql/nvme_strom.c:870-940).  Without a PostgreSQL server these are the
on-disk structures that decision reads:

  * visibility map ``<relfilenode>_vm``: pages of a 24-byte page header
    followed by 2 bits per heap block (bit 0 all-visible, bit 1 all-frozen),
    ``(BLCKSZ - 24) * 4`` heap blocks per map page (visibilitymap.c);
  * commit log ``pg_xact``: 2 bits per transaction id (0 in progress,
    1 committed, 2 aborted, 3 sub-committed);
  * ``pg_subtrans``: the parent of each subtransaction xid;
  * ``pg_multixact``: offsets and members (a locker-only xmax deletes
    nothing; an update member decides otherwise);
  * snapshot: ``xmin``, ``xmax``, the in-progress ``xip`` / ``subxip``
    lists, and the scanning transaction's own xids and command id.

The per-tuple check itself is native (strom_pg_apply_mvcc: the rules of
HeapTupleSatisfiesMVCC, pgsql/nvme_strom.c:907-936 hands buffer-manager
tuples to it); ``model_visible`` is an independent Python transcription the
tests hold it against.  Parity with a live server is unpinned: no
PostgreSQL here, and the reference ships no page fixtures.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .. import _native as N

BLCKSZ = 8192
VM_HEADER = 24
VM_ALL_VISIBLE, VM_ALL_FROZEN = 1, 2
XACT_IN_PROGRESS, XACT_COMMITTED, XACT_ABORTED, XACT_SUBCOMMITTED = 0, 1, 2, 3


def vm_blocks_per_page(blcksz: int = BLCKSZ) -> int:
    return (blcksz - VM_HEADER) * 4


def vm_path(rel_path: str) -> str:
    return rel_path + "_vm"


def write_vm(path: str, all_visible: Sequence[bool], all_frozen: Optional[Sequence[bool]] = None,
             blcksz: int = BLCKSZ) -> None:
    av = np.asarray(all_visible, dtype=bool)
    af = np.zeros_like(av) if all_frozen is None else np.asarray(all_frozen, dtype=bool)
    bits = av.astype(np.uint8) | (af.astype(np.uint8) << 1)
    per = vm_blocks_per_page(blcksz)
    pages = []
    for p0 in range(0, max(len(bits), 1), per):
        chunk = bits[p0:p0 + per]
        pad = (-len(chunk)) % 4
        c = np.concatenate([chunk, np.zeros(pad, np.uint8)]).reshape(-1, 4)
        body = (c[:, 0] | (c[:, 1] << 2) | (c[:, 2] << 4) | (c[:, 3] << 6)).astype(np.uint8)
        page = bytearray(blcksz)
        struct.pack_into("<QHHHHHHI", page, 0, 1, 0, 0, VM_HEADER, blcksz, blcksz, blcksz | 4, 0)
        page[VM_HEADER:VM_HEADER + len(body)] = body.tobytes()
        pages.append(bytes(page))
    with open(path, "wb") as f:
        f.write(b"".join(pages))


def read_vm(path: str, nblocks: int, blcksz: int = BLCKSZ) -> Optional[np.ndarray]:
    """Per heap block: bit 0 all-visible, bit 1 all-frozen (uint8), or None
    when the relation has no visibility map (every block takes the checked
    path, as in PostgreSQL)."""
    if not os.path.exists(path):
        return None
    raw = np.fromfile(path, dtype=np.uint8)
    per = vm_blocks_per_page(blcksz)
    out = np.zeros(nblocks, dtype=np.uint8)
    for p in range(len(raw) // blcksz):
        body = raw[p * blcksz + VM_HEADER:(p + 1) * blcksz]
        bits = np.stack([(body >> s) & 3 for s in (0, 2, 4, 6)], axis=1).reshape(-1)
        lo = p * per
        n = min(per, nblocks - lo)
        if n <= 0:
            break
        out[lo:lo + n] = bits[:n]
    return out


def xid_precedes(a: int, b: int) -> bool:
    """TransactionIdPrecedes: modulo 2^32 for normal xids (>= 3), plain
    order when either is special (0 invalid, 1 bootstrap, 2 frozen)."""
    a &= 0xFFFFFFFF
    b &= 0xFFFFFFFF
    if a < 3 or b < 3:
        return a < b
    d = (a - b) & 0xFFFFFFFF
    return d >= 0x80000000


class CommitLog:
    """A window of pg_xact: 2 bits per xid (0 in progress, 1 committed,
    2 aborted, 3 sub-committed) for xids base, base + 1, ... (mod 2^32, so
    a window may straddle the wraparound)."""

    def __init__(self, nxids: int = 1 << 16, base: int = 0):
        self.base = base & 0xFFFFFFFF
        self.bits = np.zeros((nxids + 3) // 4, dtype=np.uint8)

    @property
    def nxids(self) -> int:
        return len(self.bits) * 4

    def set(self, xid: int, status: int) -> None:
        k = (xid - self.base) & 0xFFFFFFFF
        if k >= self.nxids:
            grow = np.zeros((k + 4) // 4 - len(self.bits) + 1024, dtype=np.uint8)
            self.bits = np.concatenate([self.bits, grow])
        b, sh = k >> 2, (k & 3) * 2
        self.bits[b] = (int(self.bits[b]) & ~(3 << sh)) | ((status & 3) << sh)

    def raw(self, xid: int) -> Optional[int]:
        """The 2 status bits, or None outside the window."""
        k = (xid - self.base) & 0xFFFFFFFF
        if k >= self.nxids:
            return None
        return (int(self.bits[k >> 2]) >> ((k & 3) * 2)) & 3

    def status(self, xid: int) -> int:
        if xid < 3:
            return XACT_COMMITTED if xid else XACT_ABORTED
        r = self.raw(xid)
        return XACT_IN_PROGRESS if r is None else r


class SubTrans:
    """A window of pg_subtrans: the parent xid of each xid from ``base`` (0:
    a top-level transaction)."""

    def __init__(self, nxids: int = 1 << 16, base: int = 0):
        self.base = base & 0xFFFFFFFF
        self.parent = np.zeros(nxids, dtype=np.uint32)

    def set(self, xid: int, parent: int) -> None:
        self.parent[(xid - self.base) & 0xFFFFFFFF] = parent

    def get(self, xid: int) -> Optional[int]:
        k = (xid - self.base) & 0xFFFFFFFF
        return int(self.parent[k]) if k < len(self.parent) else None


MX_FOR_KEY_SHARE, MX_FOR_SHARE, MX_FOR_NO_KEY_UPDATE, MX_FOR_UPDATE = 0, 1, 2, 3
MX_NO_KEY_UPDATE, MX_UPDATE = 4, 5
_MX_GROUPS_PER_PAGE = BLCKSZ // 20          # 4 flag bytes + 4 xids per member group


class MultiXact:
    """pg_multixact windows: offsets (member offset per multixact id from
    ``base``; one more entry, the next offset, closes the last one) and
    members in PostgreSQL's page layout — 409 groups of 4 status bytes + 4
    xids per 8 KiB page, member offsets from ``members_base``."""

    def __init__(self, base: int = 1, members_base: int = 0):
        self.base = base & 0xFFFFFFFF
        self.members_base = members_base & 0xFFFFFFFF
        self.offsets = [self.members_base]
        self.members: List[Tuple[int, int]] = []     # (xid, status)

    def add(self, members: Sequence[Tuple[int, int]]) -> int:
        """A new multixact of (xid, MultiXactStatus) members; its id."""
        mid = (self.base + len(self.offsets) - 1) & 0xFFFFFFFF
        self.members.extend((int(x), int(st)) for x, st in members)
        self.offsets.append((self.members_base + len(self.members)) & 0xFFFFFFFF)
        return mid

    def offsets_array(self) -> np.ndarray:
        return np.asarray(self.offsets, dtype=np.uint32)

    def members_pages(self) -> np.ndarray:
        n = len(self.members)
        groups = (n + 3) // 4
        pages = max(1, (groups + _MX_GROUPS_PER_PAGE - 1) // _MX_GROUPS_PER_PAGE)
        buf = np.zeros(pages * BLCKSZ, dtype=np.uint8)
        for k, (x, st) in enumerate(self.members):
            g = k // 4
            o = (g // _MX_GROUPS_PER_PAGE) * BLCKSZ + (g % _MX_GROUPS_PER_PAGE) * 20
            buf[o + k % 4] = st
            buf[o + 4 + 4 * (k % 4):o + 8 + 4 * (k % 4)] = np.frombuffer(
                struct.pack("<I", x & 0xFFFFFFFF), np.uint8)
        return buf

    def get(self, multi: int) -> Optional[List[Tuple[int, int]]]:
        k = (multi - self.base) & 0xFFFFFFFF
        if k >= len(self.offsets) - 1:
            return None
        a = (self.offsets[k] - self.members_base) & 0xFFFFFFFF
        b = (self.offsets[k + 1] - self.members_base) & 0xFFFFFFFF
        return self.members[a:b]


@dataclass
class Snapshot:
    """An MVCC snapshot: xmin, xmax, the running xids (xip) and their running
    subtransactions (subxip; ``suboverflowed`` when that list did not fit,
    so pg_subtrans maps a subxid to its top-level xid), plus the scanning
    transaction itself: its xids (top-level + subtransactions) and the
    command id the scan runs at."""
    xmin: int
    xmax: int
    xip: Sequence[int] = field(default_factory=list)
    subxip: Sequence[int] = field(default_factory=list)
    suboverflowed: bool = False
    curxids: Sequence[int] = field(default_factory=list)
    curcid: int = 0

    def sees(self, xid: int) -> bool:
        """Committed xid ``xid`` is visible to this snapshot (no subtrans
        lookups: the quick form)."""
        if xid < 3 or xid_precedes(xid, self.xmin):
            return True
        return xid_precedes(xid, self.xmax) and xid not in set(self.xip) and \
            xid not in set(self.subxip)


# infomask bits (htup_details.h)
HEAP_XMAX_KEYSHR_LOCK, HEAP_COMBOCID, HEAP_XMAX_EXCL_LOCK = 0x0010, 0x0020, 0x0040
HEAP_XMAX_LOCK_ONLY, HEAP_XMIN_COMMITTED, HEAP_XMIN_INVALID = 0x0080, 0x0100, 0x0200
HEAP_XMAX_COMMITTED, HEAP_XMAX_INVALID, HEAP_XMAX_IS_MULTI = 0x0400, 0x0800, 0x1000


class _Undecided(Exception):
    pass


def model_visible(xmin: int, xmax: int, infomask: int, cid: int, snap: Snapshot,
                  clog: Optional[CommitLog], subtrans: Optional[SubTrans] = None,
                  multi: Optional[MultiXact] = None) -> Optional[bool]:
    """HeapTupleSatisfiesMVCC written out in Python, independently of the
    native check (csrc/engine/codecs.cc): True / False, or None when the
    inputs cannot decide (a combo command id of the scanning transaction,
    an xid or multixact outside the given log windows)."""
    cur = set(snap.curxids)

    def clog_raw(x):
        r = clog.raw(x) if clog is not None else None
        if r is None:
            raise _Undecided
        return r

    def parent(x):
        p = subtrans.get(x) if subtrans is not None else None
        if p is None:
            raise _Undecided
        return p

    def committed(x):                       # TransactionIdDidCommit
        for _ in range(1024):
            if x < 3:
                return x in (1, 2)
            st = clog_raw(x)
            if st != XACT_SUBCOMMITTED:
                return st == XACT_COMMITTED
            if xid_precedes(x, snap.xmin):
                return False
            x = parent(x)
            if x == 0:
                return False
        raise _Undecided

    def running(x):                         # XidInMVCCSnapshot
        if xid_precedes(x, snap.xmin):
            return False
        if not xid_precedes(x, snap.xmax):
            return True
        if not snap.suboverflowed:
            if x in set(snap.subxip):
                return True
        else:
            top, p = x, x
            for _ in range(1024):
                if not p:
                    break
                top = p
                if xid_precedes(p, snap.xmin):
                    break
                q = parent(p)
                if q and not xid_precedes(q, p):
                    raise _Undecided
                p = q
            x = top
            if xid_precedes(x, snap.xmin):
                return False
        return x in set(snap.xip)

    def current(x):
        return x >= 3 and x in cur

    def locked_only():
        return bool(infomask & HEAP_XMAX_LOCK_ONLY) or \
            (infomask & (HEAP_XMAX_IS_MULTI | HEAP_XMAX_KEYSHR_LOCK | HEAP_XMAX_EXCL_LOCK)) == \
            HEAP_XMAX_EXCL_LOCK

    def update_xid():                       # MultiXactIdGetUpdateXid
        mem = multi.get(xmax) if multi is not None else None
        if mem is None:
            raise _Undecided
        for x, st in mem:
            if st > MX_FOR_UPDATE:
                return x
        return 0

    def own_cid():
        if infomask & HEAP_COMBOCID:
            raise _Undecided
        return cid

    try:
        if not infomask & HEAP_XMIN_COMMITTED:
            if infomask & HEAP_XMIN_INVALID:
                return False
            if current(xmin):
                c = own_cid()
                if c >= snap.curcid:
                    return False
                if infomask & HEAP_XMAX_INVALID or locked_only():
                    return True
                if infomask & HEAP_XMAX_IS_MULTI:
                    return True if not current(update_xid()) else c >= snap.curcid
                if not current(xmax):
                    return True
                return c >= snap.curcid
            if running(xmin):
                return False
            if not committed(xmin):
                return False
        elif (infomask & (HEAP_XMIN_COMMITTED | HEAP_XMIN_INVALID)) != \
                (HEAP_XMIN_COMMITTED | HEAP_XMIN_INVALID) and running(xmin):
            return False
        if infomask & HEAP_XMAX_INVALID or locked_only():
            return True
        if infomask & HEAP_XMAX_IS_MULTI:
            up = update_xid()
            if not up:
                return True
            if current(up):
                return own_cid() >= snap.curcid
            if running(up):
                return True
            return not committed(up)
        if not infomask & HEAP_XMAX_COMMITTED:
            if current(xmax):
                return own_cid() >= snap.curcid
            if running(xmax):
                return True
            return not committed(xmax)
        return running(xmax)
    except _Undecided:
        return None


def mvcc_struct(snap: Snapshot, clog: Optional[CommitLog], subtrans: Optional[SubTrans] = None,
                multi: Optional[MultiXact] = None):
    """(strom_pg_mvcc, arrays it points into — keep them alive)."""
    m = N.PgMvcc()
    keep = []

    def arr(v, dt):
        a = np.ascontiguousarray(np.asarray(list(v), dtype=dt))
        keep.append(a)
        return a.ctypes.data if len(a) else None
    m.xmin, m.xmax = snap.xmin & 0xFFFFFFFF, snap.xmax & 0xFFFFFFFF
    m.xip, m.nxip = arr(snap.xip, np.uint32), len(snap.xip)
    m.subxip, m.nsubxip = arr(snap.subxip, np.uint32), len(snap.subxip)
    m.suboverflowed = int(bool(snap.suboverflowed))
    m.curxids, m.ncurxids = arr(snap.curxids, np.uint32), len(snap.curxids)
    m.curcid = snap.curcid
    if clog is not None:
        keep.append(clog.bits)
        m.clog, m.clog_n, m.clog_base = clog.bits.ctypes.data, clog.nxids, clog.base
    if subtrans is not None:
        keep.append(subtrans.parent)
        m.subtrans, m.subtrans_n = subtrans.parent.ctypes.data, len(subtrans.parent)
        m.subtrans_base = subtrans.base
    if multi is not None:
        off, mem = multi.offsets_array(), multi.members_pages()
        keep += [off, mem]
        m.mx_offsets, m.mx_base, m.mx_n = off.ctypes.data, multi.base, len(off) - 1
        m.mx_members, m.mxm_n, m.mxm_base = mem.ctypes.data, len(multi.members), multi.members_base
    return m, keep


def native_visible(tuple_header: bytes, snap: Snapshot, clog: Optional[CommitLog],
                   subtrans: Optional[SubTrans] = None,
                   multi: Optional[MultiXact] = None) -> Optional[bool]:
    """The native check of one tuple header (strom_pg_tuple_visible)."""
    import ctypes as C
    m, keep = mvcc_struct(snap, clog, subtrans, multi)
    hdr = np.frombuffer(bytes(tuple_header[:24]).ljust(24, b"\0"), np.uint8).copy()
    r = N.lib().strom_pg_tuple_visible(hdr.ctypes.data, C.byref(m))
    return None if r < 0 else bool(r)


def apply_snapshot(page: np.ndarray, snap: Snapshot, clog: Optional[CommitLog],
                   blkno: Optional[int] = None, subtrans: Optional[SubTrans] = None,
                   multi: Optional[MultiXact] = None,
                   recheck: Optional[List[int]] = None) -> int:
    """Mark the tuples of one heap page (writable uint8 array) that ``snap``
    must not see as LP_UNUSED; returns how many.  Tuples the inputs cannot
    decide are kept, their line numbers appended to ``recheck``.  With
    ``blkno`` the page checksum is verified first (as ReadBuffer does) and,
    when it was valid, re-stamped after the edit, so a later checksum pass
    still accepts the page; a corrupt page keeps its bad checksum."""
    import ctypes as C
    ck_ok = False
    if blkno is not None:
        from .pgpage import checksum
        stored = int(page[8]) | (int(page[9]) << 8)
        ck_ok = checksum(page.tobytes(), blkno) == stored
    m, keep = mvcc_struct(snap, clog, subtrans, multi)
    rc_lines = np.zeros(len(page) // 4, dtype=np.uint16)
    nr = C.c_uint32(0)
    rc = N.lib().strom_pg_apply_mvcc(page.ctypes.data, len(page), C.byref(m),
                                     rc_lines.ctypes.data, len(rc_lines), C.byref(nr))
    if rc < 0:
        raise ValueError("not a heap page")
    if recheck is not None:
        recheck.extend(int(x) for x in rc_lines[:min(nr.value, len(rc_lines))])
    if rc and ck_ok:
        from .pgpage import checksum
        c = checksum(page.tobytes(), blkno)
        page[8], page[9] = c & 0xFF, c >> 8
    return int(rc)


def read_check_pages(fd: int, blocks: np.ndarray, stage: np.ndarray, snap: Snapshot,
                     clog: Optional[CommitLog], relseg_blocks: int = 0,
                     verify_checksum: bool = False, subtrans: Optional[SubTrans] = None,
                     multi: Optional[MultiXact] = None, blcksz: int = BLCKSZ
                     ) -> Tuple[int, np.ndarray]:
    """The host ("buffer manager") leg for blocks checked on the CPU, native
    (strom_pg_read_check_pages): each block is read into ``stage`` (writable
    uint8, len(blocks) * blcksz, page i at i * blcksz), its checksum verified
    first with ``verify_checksum``, and the tuples ``snap`` must not see
    marked LP_UNUSED.  Returns (tuples removed, per-block recheck flags)."""
    blocks = np.ascontiguousarray(np.asarray(blocks, dtype=np.uint32))
    n = len(blocks)
    if stage.dtype != np.uint8 or stage.size < n * blcksz or not stage.flags.c_contiguous:
        raise ValueError("stage must be a contiguous uint8 array of len(blocks) pages")
    m, keep = mvcc_struct(snap, clog, subtrans, multi)
    flags = np.zeros(max(n, 1), dtype=np.uint8)
    import ctypes as C
    r = N.lib().strom_pg_read_check_pages(fd, blocks.ctypes.data if n else None, n, relseg_blocks,
                                          blcksz, stage.ctypes.data, C.byref(m),
                                          1 if verify_checksum else 0, flags.ctypes.data)
    if r < 0:
        raise OSError(-r, os.strerror(-r))
    return int(r), flags[:n]
