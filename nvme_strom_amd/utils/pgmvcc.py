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
  * snapshot: ``xmin``, ``xmax`` and the in-progress ``xip`` list.

The per-tuple check itself is native (strom_pg_apply_snapshot).  Parity with
a live server is unpinned: no PostgreSQL here, and the reference ships no
page fixtures.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import Optional, Sequence

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


class CommitLog:
    """pg_xact-shaped commit log: 2 bits per xid."""

    def __init__(self, nxids: int = 1 << 16):
        self.bits = np.zeros((nxids + 3) // 4, dtype=np.uint8)

    @property
    def nxids(self) -> int:
        return len(self.bits) * 4

    def set(self, xid: int, status: int) -> None:
        if xid >= self.nxids:
            grow = np.zeros((xid + 4) // 4 - len(self.bits) + 1024, dtype=np.uint8)
            self.bits = np.concatenate([self.bits, grow])
        b, sh = xid >> 2, (xid & 3) * 2
        self.bits[b] = (int(self.bits[b]) & ~(3 << sh)) | ((status & 3) << sh)

    def status(self, xid: int) -> int:
        if xid < 3:
            return XACT_COMMITTED if xid else XACT_ABORTED
        if xid >= self.nxids:
            return XACT_IN_PROGRESS
        return (int(self.bits[xid >> 2]) >> ((xid & 3) * 2)) & 3


@dataclass
class Snapshot:
    xmin: int
    xmax: int
    xip: Sequence[int] = field(default_factory=list)

    def sees(self, xid: int) -> bool:
        if xid < 3 or xid < self.xmin:
            return True
        return xid < self.xmax and xid not in set(self.xip)


def apply_snapshot(page: np.ndarray, snap: Snapshot, clog: Optional[CommitLog],
                   blkno: Optional[int] = None) -> int:
    """Mark the tuples of one heap page (writable uint8 array) that ``snap``
    must not see as LP_UNUSED; returns how many.  With ``blkno`` the page
    checksum is verified first (as ReadBuffer does) and, when it was valid,
    re-stamped after the edit, so a later checksum pass still accepts the
    page; a corrupt page keeps its bad checksum."""
    ck_ok = False
    if blkno is not None:
        from .pgpage import checksum
        stored = int(page[8]) | (int(page[9]) << 8)
        ck_ok = checksum(page.tobytes(), blkno) == stored
    xip = np.asarray(list(snap.xip), dtype=np.uint32)
    cb = clog.bits if clog is not None else None
    rc = N.lib().strom_pg_apply_snapshot(
        page.ctypes.data, len(page), snap.xmin, snap.xmax,
        xip.ctypes.data if len(xip) else None, len(xip),
        cb.ctypes.data if cb is not None else None, clog.nxids if clog is not None else 0)
    if rc < 0:
        raise ValueError("not a heap page")
    if rc and ck_ok:
        from .pgpage import checksum
        c = checksum(page.tobytes(), blkno)
        page[8], page[9] = c & 0xFF, c >> 8
    return int(rc)
