"""PostgreSQL heap-relation scan fed by the engine — the MI355X rendition of
the reference's ``pgsql/`` CustomScan provider.

Reference map (pgsql/nvme_strom.c):
  * GUCs ``nvme_strom.enabled/chunk_size/buffer_size/seq_page_cost/
    debug_no_threshold`` (:1270-1324)            -> :class:`ScanConfig`
  * planner threshold (RAM - shared_buffers)*2/3 + shared_buffers
    (:1258-1268) and cost (:398-467)              -> :func:`use_strom`, :func:`scan_cost`
  * tablespace capability cache (:192-295)        -> :class:`TablespaceCache`
  * parallel block cursor in DSM (:90-104, :1181-1233) -> :class:`ParallelCursor`
    (threads of one process) and :class:`SharedCursor` (a shared-memory
    segment + native atomics: participants in separate processes)
  * planner hook set_rel_pathlist_hook -> add_path(CustomPath) with the
    threshold and cost model (:502-580)             -> :func:`plan_scan`
  * chunk ring + load + tuple iteration (:852-1123) -> :class:`HeapRelationScan`
  * visibility-map routing (:870-940): with a snapshot, all-visible blocks
    are taken unchecked and every tuple of the others is checked against
    the snapshot, pg_xact, pg_subtrans and pg_multixact.  The reference reads
    those blocks through the buffer manager and checks them on the CPU; here
    every block is read SSD->HBM and the scan kernel runs the check
    (ScanConfig.mvcc_device, heapscan.hip mvcc_visible) for the pages the VM
    flags, so a relation that is not all-visible scans at the same rate.
    ``mvcc_device=False`` keeps the reference's split (native
    strom_pg_read_check_pages: pread + checksum + in-place LP_UNUSED)
  * ExecReScanNVMEStrom cursor reset (:1168-1176)  -> :meth:`ParallelCursor.rescan`;
    the reference persists no scan state, :class:`ResumableScan` adds
    block-range checkpoints so an interrupted scan resumes where it stopped

The ring lives in HBM: each chunk of blocks is read with MEMCPY_SSD2GPU
(``relseg_sz`` = RELSEG_SIZE maps block numbers to 1 GiB segment files) and
scanned by the GPU heap-page kernel (header check, optional checksum,
visibility hints, predicate, compaction) — no per-tuple CPU loop.  Blocks
served from the page cache land at the chunk's tail; the kernel does not
care about order, and item ids are mapped back through the landed block
numbers.  ``cpu_scan`` is the reference-shaped path (SSD2RAM into a DMA
buffer + host tuple walk) used as the parity baseline.
"""
from __future__ import annotations

import json
import os
import threading
import time
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Any

import numpy as np
import torch

from .. import api
from ..ops.heapscan import (PAGE_RECHECK, DeviceMvcc, Program, heap_project_many, heap_scan,
                            heap_scan2)
from ..tensor import FileReader, HbmBuffer, host_buffer
from ..utils import pgmvcc, pgpage, pgtuple
from ..utils.pgmvcc import CommitLog, MultiXact, Snapshot, SubTrans

BLCKSZ = 8192
RELSEG_SIZE = 131072          # blocks per segment file (1 GiB)


@dataclass
class ScanConfig:
    enabled: bool = True
    chunk_size: int = 32 << 20
    buffer_size: int = 256 << 20
    seq_page_cost: float = 0.25          # DEFAULT_SEQ_PAGE_COST / 4
    debug_no_threshold: bool = False
    verify_checksum: bool = False
    skip_invisible: bool = True
    # MVCC mode: with a snapshot, blocks route by the visibility map (all-
    # visible -> DMA, unchecked; others -> host read + per-tuple snapshot
    # check); without one, the GPU applies hint bits / PD_ALL_VISIBLE
    snapshot: Optional[Snapshot] = None
    clog: Optional[CommitLog] = None
    # the rest of HeapTupleSatisfiesMVCC's inputs: pg_subtrans (sub-committed
    # xids, overflowed snapshots) and pg_multixact (multixact xmax)
    subtrans: Optional[SubTrans] = None
    multixact: Optional[MultiXact] = None
    # where the snapshot check runs: True (default) on the GPU — every block
    # is read SSD->HBM and the scan kernel checks the tuples of the blocks
    # the VM does not call all-visible (ops.heapscan.DeviceMvcc); False: the
    # reference's split, those blocks read and checked on the host
    # (native strom_pg_read_check_pages) and copied in after the DMA blocks
    mvcc_device: bool = True

    def validate(self) -> None:
        if self.chunk_size % BLCKSZ or self.buffer_size % self.chunk_size:
            raise ValueError("chunk_size must be a multiple of BLCKSZ and divide buffer_size")


def strom_threshold(ram_bytes: int, shared_buffers: int) -> int:
    return (ram_bytes - shared_buffers) * 2 // 3 + shared_buffers


def use_strom(rel_bytes: int, ram_bytes: int, shared_buffers: int, cfg: ScanConfig,
              tablespace_ok: bool) -> bool:
    if not cfg.enabled or not tablespace_ok:
        return False
    return cfg.debug_no_threshold or rel_bytes >= strom_threshold(ram_bytes, shared_buffers)


def scan_cost(pages: int, cfg: ScanConfig, parallel_workers: int = 0,
              cpu_tuple_cost: float = 0.01, tuples: int = 0) -> float:
    divisor = 1.0 + min(parallel_workers, 4) if parallel_workers else 1.0
    return (cfg.seq_page_cost * pages + cpu_tuple_cost * tuples) / divisor


@dataclass
class ScanPlan:
    path: str                    # "nvme_strom" or "seqscan"
    cost: float
    workers: int
    seqscan_cost: float
    reason: str

    def explain(self) -> str:
        node = "Custom Scan (NVMEStrom)" if self.path == "nvme_strom" else "Seq Scan"
        par = f" (parallel workers={self.workers})" if self.workers else ""
        return f"{node}{par}  (cost=0.00..{self.cost:.2f})  -- {self.reason}"


def plan_scan(rel_bytes: int, ntuples: int, ram_bytes: int, shared_buffers: int,
              cfg: Optional[ScanConfig] = None, tablespace_ok: bool = True,
              parallel_workers: int = 0, seq_page_cost: float = 1.0,
              cpu_tuple_cost: float = 0.01) -> ScanPlan:
    """The planner hook's decision (nvmestrom_add_scan_path,
    pgsql/nvme_strom.c:502-543): offer the strom path only for relations
    on an NVMe-capable tablespace above the threshold, cost it with
    ``seq_page_cost`` (divided for parallel plans, :398-467) and keep it
    when it beats the ordinary sequential scan."""
    cfg = cfg or ScanConfig()
    pages = (rel_bytes + BLCKSZ - 1) // BLCKSZ
    seq = seq_page_cost * pages + cpu_tuple_cost * ntuples
    if not use_strom(rel_bytes, ram_bytes, shared_buffers, cfg, tablespace_ok):
        why = ("disabled" if not cfg.enabled else "tablespace not on NVMe" if not tablespace_ok
               else f"below threshold {strom_threshold(ram_bytes, shared_buffers)} bytes")
        return ScanPlan("seqscan", seq, 0, seq, why)
    cost = scan_cost(pages, cfg, parallel_workers, cpu_tuple_cost, ntuples)
    if cost < seq:
        return ScanPlan("nvme_strom", cost, parallel_workers, seq, "cheaper than seqscan")
    return ScanPlan("seqscan", seq, 0, seq, "seqscan is cheaper")


class TablespaceCache:
    """CHECK_FILE per tablespace directory, cached; invalidate on change."""

    def __init__(self):
        self._c: Dict[str, bool] = {}
        self._lock = threading.Lock()

    def can_use(self, directory: str) -> bool:
        with self._lock:
            if directory in self._c:
                return self._c[directory]
        ok = False
        try:
            fd = os.open(directory, os.O_RDONLY)
            try:
                ok = api.check_file(fd).support_dma64
            finally:
                os.close(fd)
        except (OSError, api.StromError):
            ok = False
        with self._lock:
            self._c[directory] = ok
        return ok

    def invalidate(self, directory: Optional[str] = None) -> None:
        with self._lock:
            if directory is None:
                self._c.clear()
            else:
                self._c.pop(directory, None)


class ParallelCursor:
    """Shared block cursor (pg_atomic_fetch_add_u64 on nsp_cblock)."""

    def __init__(self, nblocks: int, start: int = 0):
        self.nblocks = nblocks       # end of the claimable range
        self.start = start
        self._next = start
        self._lock = threading.Lock()

    def claim(self, n: int, boundary: int = 0) -> Tuple[int, int]:
        """Claim up to ``n`` blocks, never crossing a multiple of ``boundary``."""
        with self._lock:
            lo = self._next
            hi = min(self.nblocks, lo + n)
            if boundary:
                hi = min(hi, (lo // boundary + 1) * boundary)
            self._next = hi
            return lo, hi - lo

    def rescan(self) -> None:
        with self._lock:
            self._next = self.start


class SharedCursor:
    """Cross-process block cursor + scan counters in a shared-memory segment
    (the reference's NVMEStromParallelDesc in DSM: nsp_cblock claimed with
    pg_atomic_fetch_add_u64, per-scan counters; pgsql/nvme_strom.c:90-104,
    :1181-1233).  The leader creates it; workers attach by name.  Claims use
    a native compare-and-swap, so they never cross a ``boundary`` (segment
    file) and no block is handed out twice across processes."""

    MAGIC = 0x53545243555253  # "STRCURS"
    FIELDS = ("magic", "nblocks", "start", "next") + ("pages", "bad_pages", "nr_ram", "nr_ssd",
                                                       "nr_dma_submit", "nr_dma_blocks",
                                                       "chunks", "tuples")

    def __init__(self, name: str, nblocks: int = 0, start: int = 0, create: bool = False):
        import mmap as _mmap
        self.name = name
        self.path = f"/dev/shm/nvme-strom-scan.{name}"
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(self.path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, 8 * len(self.FIELDS))
            self._mm = _mmap.mmap(fd, 8 * len(self.FIELDS))
        finally:
            os.close(fd)
        self._a = np.frombuffer(self._mm, dtype=np.uint64)
        self._lib = api.N.lib()
        if create:
            self._a[:] = 0
            self._a[1], self._a[2], self._a[3] = nblocks, start, start
            self._a[0] = self.MAGIC
        elif int(self._a[0]) != self.MAGIC:
            raise ValueError(f"{self.path}: not a scan cursor")
        self.owner = create

    def _addr(self, i: int) -> int:
        return self._a.ctypes.data + 8 * i

    @property
    def nblocks(self) -> int:
        return int(self._a[1])

    def claim(self, n: int, boundary: int = 0) -> Tuple[int, int]:
        end = self.nblocks
        while True:
            lo = int(self._lib.strom_atomic_load_u64(self._addr(3)))
            if lo >= end:
                return lo, 0
            hi = min(end, lo + n)
            if boundary:
                hi = min(hi, (lo // boundary + 1) * boundary)
            if self._lib.strom_atomic_cas_u64(self._addr(3), lo, hi):
                return lo, hi - lo

    def rescan(self) -> None:
        self._a[3] = self._a[2]

    def add(self, r: "ScanResult") -> None:
        for i, k in enumerate(self.FIELDS[4:], start=4):
            v = r.ntuples if k == "tuples" else int(getattr(r, k))
            if v:
                self._lib.strom_atomic_fetch_add_u64(self._addr(i), v)

    def counters(self) -> Dict[str, int]:
        return {k: int(self._lib.strom_atomic_load_u64(self._addr(i)))
                for i, k in enumerate(self.FIELDS[4:], start=4)}

    def close(self, unlink: Optional[bool] = None) -> None:
        if self._mm is not None:
            self._a = None
            self._mm.close()
            self._mm = None
        if self.owner if unlink is None else unlink:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class Relation:
    """A heap relation stored as PostgreSQL segment files: path, path.1, ...
    plus its visibility-map fork ``path_vm`` when present."""

    def __init__(self, path: str, relseg_size: int = RELSEG_SIZE):
        self.path = path
        self.relseg_size = relseg_size
        self.segments: List[str] = []
        k = 0
        while True:
            p = path if k == 0 else f"{path}.{k}"
            if not os.path.exists(p):
                break
            self.segments.append(p)
            k += 1
        if not self.segments:
            raise FileNotFoundError(path)
        sizes = [os.path.getsize(p) for p in self.segments]
        self.nblocks = sum(s // BLCKSZ for s in sizes)
        self.vm = pgmvcc.read_vm(pgmvcc.vm_path(path), self.nblocks)

    def all_visible(self, lo: int, n: int) -> np.ndarray:
        """VM all-visible bits of blocks [lo, lo+n) (all False without a VM)."""
        if self.vm is None:
            return np.zeros(n, dtype=bool)
        return (self.vm[lo:lo + n] & pgmvcc.VM_ALL_VISIBLE).astype(bool)

    @staticmethod
    def write(path: str, data: bytes, relseg_size: int = RELSEG_SIZE,
              all_visible: Optional[Sequence[bool]] = None) -> "Relation":
        seg = relseg_size * BLCKSZ
        for k, lo in enumerate(range(0, len(data), seg)):
            p = path if k == 0 else f"{path}.{k}"
            with open(p, "wb") as f:
                f.write(data[lo:lo + seg])
                f.flush()
                os.fsync(f.fileno())
        if all_visible is not None:
            pgmvcc.write_vm(pgmvcc.vm_path(path), all_visible)
        return Relation(path, relseg_size)


@dataclass
class ScanResult:
    items: np.ndarray            # uint64 (blkno << 16 | lineno), sorted
    pages: int = 0
    bad_pages: int = 0
    seconds: float = 0.0
    nr_ram: int = 0
    nr_ssd: int = 0
    # the per-scan counters the reference kept in its DSM segment
    # (pgsql/nvme_strom.c:96-102) but never displayed (empty
    # ExplainNVMEStrom, :1238-1242)
    nr_dma_submit: int = 0
    nr_dma_blocks: int = 0
    chunks: int = 0
    workers: int = 1
    # per participant: (first block, item pointers) of every chunk, merged
    # in block order by HeapRelationScan.run
    chunk_items: list = field(default_factory=list, repr=False)
    # MVCC mode: blocks that took the checked (host) path, tuples it removed
    nr_checked: int = 0
    removed: int = 0
    # qualifier-list scans: the projected column of every item (numpy int64 /
    # float64, or a list of bytes for a varlena column) and its validity (0
    # NULL, 1 value, 2 compressed / out-of-line: the executor detoasts it)
    values: Optional[Any] = None
    valid: Optional[np.ndarray] = None
    # blocks holding tuples a text qualifier could not decide on the GPU
    # (compressed / TOAST values): the executor re-evaluates those blocks
    recheck_blocks: List[int] = field(default_factory=list)
    # every projected column: {name: (values, valid)} as values / valid
    # (a numeric column's values are decimal.Decimal)
    columns: Dict[str, tuple] = field(default_factory=dict)

    @property
    def ntuples(self) -> int:
        return len(self.items)

    def add_io(self, r) -> None:
        self.nr_ram += r.nr_ram
        self.nr_ssd += r.nr_ssd
        self.nr_dma_submit += r.nr_dma_submit
        self.nr_dma_blocks += r.nr_dma_blocks
        self.chunks += 1

    def merge(self, parts: List["ScanResult"]) -> None:
        for p in parts:
            self.pages += p.pages
            self.bad_pages += p.bad_pages
            self.nr_ram += p.nr_ram
            self.nr_ssd += p.nr_ssd
            self.nr_dma_submit += p.nr_dma_submit
            self.nr_dma_blocks += p.nr_dma_blocks
            self.chunks += p.chunks
            self.nr_checked += p.nr_checked
            self.removed += p.removed
            self.recheck_blocks += p.recheck_blocks
        self.recheck_blocks.sort()

    def explain(self) -> str:
        """EXPLAIN ANALYZE-style summary of the scan's I/O split and rates."""
        blocks = self.nr_ram + self.nr_ssd
        avg_kib = 0.5 * self.nr_dma_blocks / self.nr_dma_submit if self.nr_dma_submit else 0.0
        mib = self.pages * BLCKSZ / (1 << 20)
        rate = mib / self.seconds if self.seconds > 0 else 0.0
        lines = [
            f"Custom Scan (NVMEStrom)  (actual rows={self.ntuples} pages={self.pages} workers={self.workers})",
            f"  Blocks: ssd2dev={self.nr_ssd} ram2dev={self.nr_ram}"
            + (f" ({100.0 * self.nr_ram / blocks:.1f}% page cache)" if blocks else ""),
            f"  DMA: submits={self.nr_dma_submit} sectors={self.nr_dma_blocks} avg={avg_kib:.1f} KiB chunks={self.chunks}",
            f"  Bad pages: {self.bad_pages}",
            f"  Visibility: checked blocks={self.nr_checked} tuples removed={self.removed}",
            f"  Time: {self.seconds * 1e3:.2f} ms ({rate:.1f} MiB/s)",
        ]
        return "\n".join(lines)


class HeapRelationScan:
    """GPU scan of a relation with ``workers`` parallel participants."""

    def __init__(self, rel: Relation, cfg: Optional[ScanConfig] = None, device=None,
                 attr_off: int = -1, attr_width: int = 8, lo: int = -(1 << 63),
                 hi: int = (1 << 63) - 1, desc=None, quals=None, project=None):
        """``attr_off``..``hi``: the fixed-offset int predicate of the round-1
        kernel.  ``desc`` (utils.pgtuple.TupleDesc) + ``quals`` (a list of
        pgtuple.Qual, ANDed, and pgtuple.Or clauses: CNF) + optional
        ``project`` column or list of columns: every tuple is deformed on the
        GPU and the qualifier list evaluated there, as the reference's
        ExecScan does on the CPU (pgsql/nvme_strom.c:1137-1143)."""
        self.rel = rel
        self.cfg = cfg or ScanConfig()
        self.cfg.validate()
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.pred = dict(attr_off=attr_off, attr_width=attr_width, lo=lo, hi=hi)
        if (quals is not None or project is not None) and desc is None:
            raise ValueError("quals / project need a tuple descriptor (desc)")
        if desc is not None and attr_off >= 0:
            raise ValueError("a fixed-offset predicate and a qualifier list are exclusive")
        self.desc, self.quals, self.project = desc, list(quals or []), project
        self._cols = ([] if project is None else [project] if isinstance(project, (str, int))
                      else list(project))
        # compiled once per scan object (checked and uploaded per chunk)
        self._prog = Program(desc, self.quals) if desc is not None else None
        # idle participant resources (session, HBM ring, readers, pinned
        # write-back buffers), reused by later runs: allocating and pinning
        # them per run cost more than the scan of a GiB-sized relation.
        # Entries are keyed by the configuration they were sized for, and
        # released by close() / the context manager / garbage collection
        # (weakref.finalize: a scan object that is simply dropped leaks
        # nothing).
        self._pool: List[tuple] = []
        self._pool_lock = threading.Lock()
        self._finalizer = weakref.finalize(self, HeapRelationScan._drain, self._pool,
                                           self._pool_lock)

    def _host_mvcc(self) -> bool:
        return self.cfg.snapshot is not None and not self.cfg.mvcc_device

    def _pool_key(self) -> tuple:
        c = self.cfg
        return (c.buffer_size, c.chunk_size, self._host_mvcc(), str(self.device))

    def _acquire(self) -> tuple:
        key = self._pool_key()
        stale = []
        with self._pool_lock:
            while self._pool:
                k, rs = self._pool.pop()
                if k == key:
                    break
                stale.append(rs)
            else:
                rs = None
        for old in stale:                     # sized for another configuration
            self._free(old)
        if rs is not None:
            return rs
        cfg = self.cfg
        per_chunk = cfg.chunk_size // BLCKSZ
        nslots = cfg.buffer_size // cfg.chunk_size
        sess = api.Session()
        hb = HbmBuffer(cfg.buffer_size, self.device, sess=sess)
        readers = [FileReader(p, BLCKSZ, self.rel.relseg_size, per_chunk, sess) for p in self.rel.segments]
        wbs = [host_buffer(cfg.chunk_size) for _ in range(nslots)]
        # checked-path pages (MVCC mode) are staged here, then copied to HBM
        # right after the chunk's DMA blocks
        cpu_bufs = [host_buffer(cfg.chunk_size) for _ in range(nslots)] if self._host_mvcc() else []
        return sess, hb, readers, wbs, cpu_bufs

    def _release(self, rs: tuple) -> None:
        with self._pool_lock:
            self._pool.append((self._pool_key(), rs))

    @staticmethod
    def _free(rs: tuple) -> None:
        sess, hb, readers, _, _ = rs
        for r in readers:
            r.close()
        hb.close()
        sess.close()

    @staticmethod
    def _drain(pool: list, lock) -> None:
        with lock:
            items = list(pool)
            pool.clear()
        for _, rs in items:
            HeapRelationScan._free(rs)

    def close(self) -> None:
        """Release the pooled participant resources."""
        self._drain(self._pool, self._pool_lock)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def run(self, workers: int = 1, blocks: Optional[Tuple[int, int]] = None,
            cursor=None) -> ScanResult:
        """Scan all blocks, or the block range ``[b0, b1)`` given as ``blocks``,
        with ``workers`` participant threads.  ``cursor`` (e.g. a
        :class:`SharedCursor` other processes also claim from) replaces the
        private one: this process then scans its share."""
        b0, b1 = _block_range(blocks, self.rel.nblocks)
        if cursor is None:
            cursor = ParallelCursor(b1, start=b0)
        # the snapshot check's inputs, uploaded once per run for every
        # participant's launches (they may change between runs)
        c = self.cfg
        self._dmvcc = (DeviceMvcc(c.snapshot, c.clog, c.subtrans, c.multixact, self.device)
                       if c.snapshot is not None and c.mvcc_device else None)
        results: List[ScanResult] = []
        errors: List[BaseException] = []
        t0 = time.perf_counter()

        def participant():
            try:
                results.append(self._participant(cursor))
            except BaseException as e:  # pragma: no cover
                errors.append(e)

        ths = [threading.Thread(target=participant) for _ in range(workers)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        if errors:
            raise errors[0]
        # each chunk is a contiguous block range with its items in order:
        # ordering the chunks by first block orders every item (no sort of
        # the items themselves: that was most of a GiB-scale scan's host time)
        chunks = sorted((c for r in results for c in r.chunk_items), key=lambda c: c[0])
        items = np.concatenate([c[1] for c in chunks]) if chunks else np.zeros(0, np.uint64)
        out = ScanResult(items, seconds=time.perf_counter() - t0, workers=workers)
        for j, col in enumerate(self._cols):
            vals = [c[2][j] for c in chunks]
            if not vals:
                values = [] if self.desc.attlen[self.desc.attno(col)] < 0 else np.zeros(0)
            elif isinstance(vals[0], list):
                values = [v for part in vals for v in part]
            else:
                values = np.concatenate(vals)
            valid = (np.concatenate([c[3][j] for c in chunks]) if chunks
                     else np.zeros(0, np.uint8))
            out.columns[col] = (values, valid)
        if self._cols and not isinstance(self.project, (list, tuple)):
            out.values, out.valid = out.columns[self._cols[0]]
        out.merge(results)
        return out

    def _participant(self, cursor) -> ScanResult:
        cfg = self.cfg
        mvcc = self._host_mvcc()          # the host leg of the VM split
        per_chunk = cfg.chunk_size // BLCKSZ
        nslots = cfg.buffer_size // cfg.chunk_size
        rs = self._acquire()
        sess, hb, readers, wbs, cpu_bufs = rs
        ring: List[Optional[tuple]] = [None] * nslots
        found: List[Tuple[int, np.ndarray]] = []    # (first block, item pointers)
        st = ScanResult(np.zeros(0, np.uint64))
        k = 0
        try:
            while True:
                slot = k % nslots
                if ring[slot] is not None:
                    self._consume(ring[slot], hb, readers, found, st)
                    ring[slot] = None
                # a chunk never spans two segment files
                lo, n = cursor.claim(per_chunk, boundary=self.rel.relseg_size)
                if n == 0:
                    break
                seg = lo // self.rel.relseg_size
                ids = np.arange(lo, lo + n, dtype=np.uint32)
                cpu_ids = ids[:0]
                if mvcc:
                    av = self.rel.all_visible(lo, n)
                    ids, cpu_ids = ids[av], ids[~av]
                res, landed = None, ids[:0]
                if len(ids):
                    res, landed = readers[seg].submit(hb, slot * cfg.chunk_size, ids,
                                                      wb=wbs[slot])
                if len(cpu_ids):
                    st.removed += self._checked_pages(readers[seg].fd, cpu_ids, cpu_bufs[slot], st)
                    st.nr_checked += len(cpu_ids)
                    at = slot * cfg.chunk_size + len(ids) * BLCKSZ
                    nb = len(cpu_ids) * BLCKSZ
                    hb.tensor[at:at + nb].copy_(cpu_bufs[slot][:nb], non_blocking=True)
                ring[slot] = (res, landed, slot, seg, cpu_ids)
                k += 1
            for item in ring:
                if item is not None:
                    self._consume(item, hb, readers, found, st)
        except BaseException:
            self._free(rs)          # a failed participant's reads may still be in flight
            raise
        self._release(rs)
        st.chunk_items = found
        return st

    def _checked_pages(self, fd: int, blocks: np.ndarray, stage: torch.Tensor,
                       st: "ScanResult") -> int:
        """Buffer-manager path (``mvcc_device=False``, and the host recheck
        leg): read the blocks and mark the tuples the snapshot must not see
        as unused, natively (blocks with tuples the inputs cannot decide go
        to ``st.recheck_blocks``)."""
        arr = stage.numpy() if stage.device.type == "cpu" else stage.cpu().numpy()
        c = self.cfg
        removed, rc = pgmvcc.read_check_pages(fd, blocks, arr, c.snapshot, c.clog,
                                              self.rel.relseg_size, c.verify_checksum,
                                              c.subtrans, c.multixact, BLCKSZ)
        st.recheck_blocks += [int(b) for b in blocks[rc.astype(bool)]]
        return removed

    def _consume(self, item, hb, readers, found, st: ScanResult) -> None:
        res, landed, slot, seg, cpu_ids = item
        if res is not None:
            readers[seg].finish(res)
        landed = np.concatenate([landed, cpu_ids])
        n = len(landed)
        pages = hb.tensor[slot * self.cfg.chunk_size: slot * self.cfg.chunk_size + n * BLCKSZ]
        blk = torch.from_numpy(landed.astype(np.int64).astype(np.uint32).view(np.int32)).to(pages.device)
        # MVCC mode: visibility is the snapshot's (all-visible blocks
        # unchecked, the rest checked on the device or already filtered on
        # the host): no hint-bit rule
        skip = self.cfg.skip_invisible and self.cfg.snapshot is None
        general = self.desc is not None
        dm = getattr(self, "_dmvcc", None)
        chk = None
        if dm is not None:
            # the VM's verdict per landed block: 1 = check its tuples
            vm = self.rel.vm
            chk = (np.ones(n, np.uint8) if vm is None
                   else ((vm[landed.astype(np.int64)] & pgmvcc.VM_ALL_VISIBLE) == 0).astype(np.uint8))
            st.nr_checked += int(chk.sum())
        if general:
            r = heap_scan2(pages, self.desc, self._prog, BLCKSZ,
                           verify_checksum=self.cfg.verify_checksum, skip_invisible=skip,
                           blknos=blk, mvcc=dm, mvcc_pages=chk)
        else:
            r = heap_scan(pages, BLCKSZ, verify_checksum=self.cfg.verify_checksum,
                          skip_invisible=skip, blknos=blk, mvcc=dm, mvcc_pages=chk,
                          **self.pred)
        st.removed += int(r.removed)
        # the kernel reserves output per workgroup (arbitrary order across
        # workgroups): sort the chunk's items on the GPU (page order) before
        # the copy, so chunks only need ordering by their first block
        srt, perm = torch.sort(r.items[:r.count].to(torch.int64) & 0xFFFFFFFF)
        it = srt.cpu().numpy().astype(np.uint32)
        page_idx = (it >> 16).astype(np.int64)
        lineno = (it & 0xFFFF).astype(np.uint64)
        blocks = landed.astype(np.uint64)[page_idx]
        ptrs = (blocks << np.uint64(16)) | lineno
        vals, valid = [], []
        if general and self._cols:
            # every projected column in one deform walk per tuple
            cnt = torch.tensor([r.count], dtype=torch.int32, device=pages.device)
            got = heap_project_many(pages, r.items, cnt, self.desc, self._cols, BLCKSZ,
                                    cap=max(r.count, 1))
            for col in self._cols:
                v, ok = got[col]
                v, ok = v[:r.count][perm], ok[:r.count][perm]
                valid.append(ok.cpu().numpy())
                k = self.desc.attno(col)
                if self.desc.attlen[k] < 0:
                    b = _gather_varlena(pages, v, ok)
                    if self.desc.kinds[k] == "numeric":
                        b = [pgtuple.numeric_value(x) if f == 1 else x
                             for x, f in zip(b, valid[-1].tolist())]
                    vals.append(b)
                else:
                    vals.append(v.cpu().numpy())
        if n > 1 and bool((landed[1:] < landed[:-1]).any()):
            o = np.argsort(ptrs, kind="stable")  # page-cache chunks landed at the tail
            ptrs = ptrs[o]
            valid = [x[o] for x in valid]
            vals = [[x[j] for j in o] if isinstance(x, list) else x[o] for x in vals]
        found.append((int(landed.min()) if n else 0, ptrs, vals, valid))
        status = r.page_status.cpu().numpy()
        if general or dm is not None:
            st.recheck_blocks += [int(landed[j]) for j in np.nonzero(status & PAGE_RECHECK)[0]]
        st.pages += n
        st.bad_pages += int(((status & 3) != 0).sum())
        if res is not None:
            st.add_io(res)


def _gather_varlena(pages: torch.Tensor, v: torch.Tensor, ok: torch.Tensor) -> list:
    """Bytes of projected inline varlena values ((offset << 32 | length) into
    ``pages``), gathered on the device into one packed copy; b"" where the
    value is NULL or not inline."""
    n = v.numel()
    if n == 0:
        return []
    inline = ok == 1
    lens = torch.where(inline, v & 0xFFFFFFFF, torch.zeros_like(v))
    offs = torch.where(inline, v >> 32, torch.zeros_like(v))
    ends = torch.cumsum(lens, 0)
    total = int(ends[-1].item())
    starts = ends - lens
    if total:
        row = torch.repeat_interleave(torch.arange(n, device=v.device), lens)
        pos = torch.arange(total, device=v.device) - starts[row] + offs[row]
        packed = pages[pos].cpu().numpy().tobytes()
    else:
        packed = b""
    s, e = starts.cpu().numpy(), ends.cpu().numpy()
    return [packed[a:b] for a, b in zip(s.tolist(), e.tolist())]


def _block_range(blocks: Optional[Tuple[int, int]], nblocks: int) -> Tuple[int, int]:
    if blocks is None:
        return 0, nblocks
    b0, b1 = int(blocks[0]), min(int(blocks[1]), nblocks)
    if b0 < 0 or b0 > b1:
        raise ValueError(f"bad block range {blocks} for {nblocks} blocks")
    return b0, b1


def cpu_scan(rel: Relation, cfg: Optional[ScanConfig] = None, attr_off: int = -1,
             attr_width: int = 8, lo: int = -(1 << 63), hi: int = (1 << 63) - 1,
             blocks: Optional[Tuple[int, int]] = None, desc=None, quals=None,
             project=None) -> ScanResult:
    """Reference-shaped path: SSD2RAM into a NUMA DMA buffer, host tuple walk
    (with ``desc`` / ``quals`` / ``project``: the host deformer,
    utils.pgtuple.host_scan2)."""
    cfg = cfg or ScanConfig()
    general = desc is not None
    cols = [] if project is None else [project] if isinstance(project, (str, int)) else list(project)
    vals_out = [[] for _ in cols]
    valid_out = [[] for _ in cols]

    def walk(raw, blkno):
        """(item ids, statuses) of pages ``raw`` starting at block ``blkno``"""
        if not general:
            return pgpage.host_scan(raw, BLCKSZ, skip, attr_off, attr_width, lo, hi,
                                    cfg.verify_checksum, blkno)
        its, stt, pv = pgtuple.host_scan2(raw, desc, quals or [], BLCKSZ, skip,
                                          cfg.verify_checksum, blkno, cols or None)
        for row in pv if cols else ():
            for j, v in enumerate(row):
                valid_out[j].append(0 if v is None else 2 if v is pgtuple.EXT else 1)
                vals_out[j].append(b"" if v is None or v is pgtuple.EXT else v)
        for j, x in enumerate(stt):
            if x & pgtuple.PAGE_RECHECK:
                st.recheck_blocks.append(blkno + j)
        return its, stt
    mvcc = cfg.snapshot is not None
    b0, b1 = _block_range(blocks, rel.nblocks)
    per_chunk = cfg.chunk_size // BLCKSZ
    t0 = time.perf_counter()
    items: List[int] = []
    st = ScanResult(np.zeros(0, np.uint64))
    with api.alloc_dma_buffer(cfg.chunk_size) as buf:
        for seg, path in enumerate(rel.segments):
            fd = os.open(path, os.O_RDONLY)
            try:
                nblk = os.fstat(fd).st_size // BLCKSZ
                base = seg * rel.relseg_size
                first = max(0, b0 - base)
                nblk = min(nblk, b1 - base)
                for c0 in range(first, nblk, per_chunk):
                    n = min(per_chunk, nblk - c0)
                    ids = np.arange(base + c0, base + c0 + n, dtype=np.uint32)
                    cpu_ids = ids[:0]
                    if mvcc:
                        av = rel.all_visible(base + c0, n)
                        ids, cpu_ids = ids[av], ids[~av]
                    if len(ids):
                        r = api.memcpy_ssd2ram(buf.address, fd, ids, BLCKSZ, rel.relseg_size)
                        api.memcpy_wait(r.dma_task_id)
                        st.add_io(r)
                    if len(cpu_ids):
                        # buffer-manager path: page cache read + snapshot
                        # check (native), after the DMA'd blocks
                        stage = buf.array[len(ids) * BLCKSZ:(len(ids) + len(cpu_ids)) * BLCKSZ]
                        rm, rc = pgmvcc.read_check_pages(fd, cpu_ids, stage, cfg.snapshot, cfg.clog,
                                                         rel.relseg_size, cfg.verify_checksum,
                                                         cfg.subtrans, cfg.multixact, BLCKSZ)
                        st.removed += rm
                        st.recheck_blocks += [int(b) for b in cpu_ids[rc.astype(bool)]]
                    st.nr_checked += len(cpu_ids)
                    blocks_here = np.concatenate([ids, cpu_ids]).astype(np.int64)
                    # block numbers feed the checksum: scan page by page
                    # when the order is not the plain file order
                    skip = cfg.skip_invisible and not mvcc
                    raw = bytes(buf.array[:n * BLCKSZ])
                    if np.array_equal(blocks_here, np.arange(base + c0, base + c0 + n)):
                        its, status = walk(raw, base + c0)
                        items.extend(((base + c0 + (i >> 16)) << 16) | (i & 0xFFFF) for i in its)
                    else:
                        status = []
                        for j, b in enumerate(blocks_here.tolist()):
                            its, stt = walk(raw[j * BLCKSZ:(j + 1) * BLCKSZ], b)
                            items.extend((b << 16) | (i & 0xFFFF) for i in its)
                            status += stt
                    st.pages += n
                    st.bad_pages += sum(1 for s in status if s & 3)
            finally:
                os.close(fd)
    order = np.argsort(np.array(items, dtype=np.uint64), kind="stable")
    st.items = np.array(items, dtype=np.uint64)[order]
    for j, col in enumerate(cols if general else ()):
        k = desc.attno(col)
        valid = np.array(valid_out[j], dtype=np.uint8)[order]
        if desc.attlen[k] < 0:
            values = [vals_out[j][i] for i in order]
        else:
            dt = np.float64 if desc.kinds[k] == "float" else np.int64
            values = np.array([0 if isinstance(v, bytes) else v for v in vals_out[j]], dtype=dt)[order]
        st.columns[col] = (values, valid)
    if cols and not isinstance(project, (list, tuple)):
        st.values, st.valid = st.columns[cols[0]]
    st.recheck_blocks.sort()
    st.seconds = time.perf_counter() - t0
    return st


def _atomic_write(path: str, write) -> None:
    """Crash-safe replace of ``path``: unique temp file in the same directory
    (two writers never share it), fsync, rename, then fsync the directory so
    the rename itself survives a crash."""
    import tempfile
    d = os.path.dirname(os.path.abspath(path))
    fd, tmp = tempfile.mkstemp(prefix=os.path.basename(path) + ".", suffix=".tmp", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            write(f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
    dfd = os.open(d, os.O_RDONLY)
    try:
        os.fsync(dfd)
    finally:
        os.close(dfd)


class ResumableScan:
    """Checkpointed scan: the relation is scanned in block ranges of
    ``step_blocks``; after each range its qualifying items go to a file of
    their own (``<path>.r<b0>-<b1>.npy``) and then the checkpoint ``path`` (an
    .npz holding only arrays, loaded with ``allow_pickle=False``) is replaced
    with the new cursor, counters and range list.  Every write is a unique
    temp file + fsync + rename + directory fsync, so checkpoint I/O per range
    is O(range) — not O(everything so far) — and a crash leaves either the
    old or the new checkpoint.  A new instance over the same checkpoint
    continues at the first unscanned block, so each block's tuples are
    reported exactly once across interruptions.

    ``scan`` is any ``(b0, b1) -> ScanResult`` — e.g. one scan object reused
    for every range (its participant resources are pooled across runs)::

        with HeapRelationScan(rel, cfg) as hs:
            ResumableScan(lambda b0, b1: hs.run(4, blocks=(b0, b1)), ...).run()

    or the ``cpu_scan`` path.  ``key`` (required, non-empty) identifies the relation,
    predicate and scan options — :func:`scan_key` builds one; resuming a
    checkpoint written under a different key, block count or step raises
    ``ValueError``.
    """

    _COUNTERS = ("pages", "bad_pages", "nr_ram", "nr_ssd", "nr_dma_submit", "nr_dma_blocks",
                 "chunks")

    def __init__(self, scan, nblocks: int, path: str, step_blocks: int, key: str):
        if step_blocks <= 0:
            raise ValueError("step_blocks must be positive")
        if not key:
            raise ValueError("a non-empty key (relation + predicate + options) is required: "
                             "see scan_key()")
        self.scan, self.nblocks, self.path, self.step, self.key = scan, nblocks, path, step_blocks, key
        self.next_block = 0
        self.ranges: List[str] = []          # item files of the finished ranges, in order
        self.counters = dict.fromkeys(self._COUNTERS, 0)
        self.seconds = 0.0
        if os.path.exists(path):
            self._load()

    def _load(self) -> None:
        with np.load(self.path, allow_pickle=False) as z:
            meta = json.loads(bytes(z["meta"]).decode())
        if (meta["key"] != self.key or meta["nblocks"] != self.nblocks
                or meta.get("step_blocks") != self.step):
            raise ValueError(f"checkpoint {self.path} is for {meta['key']!r}/{meta['nblocks']} blocks/"
                             f"step {meta.get('step_blocks')}, not {self.key!r}/{self.nblocks}/{self.step}")
        self.next_block = int(meta["next_block"])
        self.counters.update({k: int(meta[k]) for k in self._COUNTERS})
        self.seconds = float(meta["seconds"])
        self.ranges = list(meta["ranges"])
        d = os.path.dirname(os.path.abspath(self.path))
        for name in self.ranges:
            if not os.path.exists(os.path.join(d, name)):
                raise ValueError(f"checkpoint {self.path}: range file {name} is missing")

    def _range_path(self, name: str) -> str:
        return os.path.join(os.path.dirname(os.path.abspath(self.path)), name)

    def _save_range(self, b0: int, b1: int, items: np.ndarray) -> str:
        name = f"{os.path.basename(self.path)}.r{b0}-{b1}.npy"
        _atomic_write(self._range_path(name), lambda f: np.save(f, items, allow_pickle=False))
        return name

    def _save_meta(self) -> None:
        meta = dict(self.counters, key=self.key, nblocks=self.nblocks, step_blocks=self.step,
                    next_block=self.next_block, seconds=self.seconds, ranges=self.ranges)
        blob = np.frombuffer(json.dumps(meta).encode(), np.uint8)
        _atomic_write(self.path, lambda f: np.savez(f, meta=blob))

    def items(self) -> np.ndarray:
        parts = [np.load(self._range_path(n), allow_pickle=False).astype(np.uint64)
                 for n in self.ranges]
        return np.sort(np.concatenate(parts)) if parts else np.zeros(0, np.uint64)

    @property
    def done(self) -> bool:
        return self.next_block >= self.nblocks

    def run(self, max_steps: Optional[int] = None) -> Optional[ScanResult]:
        """Scan up to ``max_steps`` ranges (all if None); returns the merged
        result once the whole relation is done, else None."""
        steps = 0
        while not self.done and (max_steps is None or steps < max_steps):
            b0 = self.next_block
            b1 = min(self.nblocks, b0 + self.step)
            r = self.scan(b0, b1)
            self.ranges.append(self._save_range(b0, b1, np.asarray(r.items, np.uint64)))
            for k in self._COUNTERS:
                self.counters[k] += int(getattr(r, k))
            self.seconds += r.seconds
            self.next_block = b1
            self._save_meta()      # the range counts only once the checkpoint names it
            steps += 1
        if not self.done:
            return None
        out = ScanResult(self.items(), seconds=self.seconds)
        for k, v in self.counters.items():
            setattr(out, k, v)
        return out

    def remove(self) -> None:
        """Delete the checkpoint and its range files (after a finished scan)."""
        for n in self.ranges:
            try:
                os.unlink(self._range_path(n))
            except FileNotFoundError:
                pass
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass


def scan_key(rel: "Relation", cfg: Optional[ScanConfig] = None, attr_off: int = -1,
             attr_width: int = 8, lo: int = -(1 << 63), hi: int = (1 << 63) - 1) -> str:
    """Checkpoint key for :class:`ResumableScan`: relation files (path, inode,
    size, mtime), predicate and the options that change the result."""
    cfg = cfg or ScanConfig()
    files = []
    for p in rel.segments:
        st = os.stat(p)
        files.append(f"{os.path.abspath(p)}:{st.st_ino}:{st.st_size}:{st.st_mtime_ns}")
    return json.dumps(dict(files=files, attr_off=attr_off, attr_width=attr_width, lo=lo, hi=hi,
                           skip_invisible=cfg.skip_invisible,
                           verify_checksum=cfg.verify_checksum), sort_keys=True)
