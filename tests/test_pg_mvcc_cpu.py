"""PostgreSQL executor semantics without a server: visibility-map routing
with per-tuple snapshot checks (pgsql/nvme_strom.c:870-940), the
cross-process block cursor in shared memory (:90-104, :1181-1233) and the
planner hook's path choice (:502-580).  Parity with a live PostgreSQL is
unpinned (no server here, no page fixtures in the reference); the rules are
checked against an independent Python model of HeapTupleSatisfiesMVCC.
"""
import os
import struct
import uuid

import numpy as np
import pytest
import torch.multiprocessing as mp

from nvme_strom_amd.models import pg_scan
from nvme_strom_amd.utils import pgmvcc, pgpage
from nvme_strom_amd.utils.pgmvcc import CommitLog, Snapshot

XMIN_C, XMIN_I, XMAX_C, XMAX_I = 0x0100, 0x0200, 0x0400, 0x0800


def test_vm_roundtrip_multi_page(tmp_path):
    n = pgmvcc.vm_blocks_per_page() + 1000          # spans two map pages
    rng = np.random.default_rng(0)
    av = rng.random(n) < 0.5
    af = av & (rng.random(n) < 0.5)
    p = str(tmp_path / "rel_vm")
    pgmvcc.write_vm(p, av, af)
    assert os.path.getsize(p) == 2 * 8192
    vm = pgmvcc.read_vm(p, n)
    assert np.array_equal(vm & 1, av.astype(np.uint8))
    assert np.array_equal((vm >> 1) & 1, af.astype(np.uint8))
    assert pgmvcc.read_vm(str(tmp_path / "none_vm"), n) is None


def _model_visible(xmin, xmax, mask, snap, clog):
    """The independent Python transcription (pgmvcc.model_visible); an
    undecidable tuple (None) is kept."""
    r = pgmvcc.model_visible(xmin, xmax, mask, 0, snap, clog)
    return True if r is None else r


def _case_tuples(rng, n, clog):
    out = []
    for i in range(n):
        xmin = int(rng.integers(3, 200))
        xmax = int(rng.choice([0, int(rng.integers(3, 200))]))
        mask = int(rng.choice([0, XMIN_C, XMIN_I, XMIN_C | XMIN_I])) | \
            int(rng.choice([0, XMAX_I, XMAX_C, 0x0080]))
        out.append((i, xmin, xmax, mask))
    return out


def test_apply_snapshot_matches_model():
    rng = np.random.default_rng(5)
    clog = CommitLog(256)
    for x in range(3, 200):
        clog.set(x, int(rng.choice([0, 1, 1, 1, 2, 3])))
    snap = Snapshot(xmin=60, xmax=150, xip=[70, 71, 99, 120])
    cases = _case_tuples(rng, 150, clog)
    tuples = [pgpage.tuple_bytes(struct.pack("<q", i), infomask=m, xmin=a, xmax=b)
              for i, a, b, m in cases]
    page = np.frombuffer(bytearray(pgpage.build_page(tuples, with_checksum=False)), np.uint8).copy()
    removed = pgmvcc.apply_snapshot(page, snap, clog)
    items, _ = pgpage.host_scan(page.tobytes(), 8192, skip_invisible=False)
    kept = {(i & 0xFFFF) - 1 for i in items}
    want = {i for i, a, b, m in cases if _model_visible(a, b, m, snap, clog)}
    assert kept == want
    assert removed == len(cases) - len(want)
    # an all-visible page is never touched
    allvis = np.frombuffer(bytearray(pgpage.build_page(tuples, with_checksum=False,
                                                       all_visible=True)), np.uint8).copy()
    assert pgmvcc.apply_snapshot(allvis, snap, clog) == 0


def _mvcc_relation(tmp_path, nblocks=24, per_page=40):
    """Blocks 0, 3, 6, ... all-visible (VM bit + PD_ALL_VISIBLE, rows with
    no hint bits); the others hold rows of mixed transaction states."""
    rng = np.random.default_rng(9)
    clog = CommitLog(512)
    for x in range(3, 400):
        clog.set(x, int(rng.choice([1, 1, 1, 2, 0])))
    snap = Snapshot(xmin=100, xmax=300, xip=[150, 151, 222])
    pages, av, want = [], [], set()
    for b in range(nblocks):
        allvis = b % 3 == 0
        tuples = []
        for j in range(per_page):
            v = b * per_page + j
            if allvis:
                xmin, xmax, mask = int(rng.integers(3, 90)), 0, 0
            else:
                xmin = int(rng.integers(3, 400))
                xmax = int(rng.choice([0, int(rng.integers(3, 400))]))
                mask = int(rng.choice([0, XMIN_C, XMIN_I])) | int(rng.choice([0, XMAX_I]))
            tuples.append(pgpage.tuple_bytes(struct.pack("<q", v), infomask=mask, xmin=xmin,
                                             xmax=xmax))
            if allvis or _model_visible(xmin, xmax, mask, snap, clog):
                want.add((b << 16) | (j + 1))
        pages.append(pgpage.build_page(tuples, blkno=b, all_visible=allvis))
        av.append(allvis)
    rel = pg_scan.Relation.write(str(tmp_path / "16384"), b"".join(pages), relseg_size=8,
                                 all_visible=av)
    return rel, snap, clog, want, sum(1 for a in av if not a)


def test_cpu_scan_vm_routing(strom, tmp_path):
    rel, snap, clog, want, nchecked = _mvcc_relation(tmp_path)
    assert len(rel.segments) == 3 and rel.vm is not None
    cfg = pg_scan.ScanConfig(chunk_size=5 * 8192, buffer_size=10 * 8192, snapshot=snap, clog=clog,
                             verify_checksum=True)
    r = pg_scan.cpu_scan(rel, cfg)
    assert set(r.items.tolist()) == want
    assert r.nr_checked == nchecked and r.bad_pages == 0
    assert r.nr_ssd + r.nr_ram == rel.nblocks - nchecked      # only all-visible blocks DMA'd
    assert "checked blocks" in r.explain()
    # without a snapshot the hint-bit rule applies instead (different set)
    r2 = pg_scan.cpu_scan(rel, pg_scan.ScanConfig(chunk_size=5 * 8192, buffer_size=10 * 8192))
    assert r2.nr_checked == 0


def _cursor_worker(name, n, boundary, q):
    try:
        c = pg_scan.SharedCursor(name)
        got = []
        while True:
            lo, k = c.claim(n, boundary)
            if k == 0:
                break
            got.append((lo, k))
            r = pg_scan.ScanResult(np.zeros(k, np.uint64), pages=k, chunks=1)
            c.add(r)
        c.close()
        q.put(got)
    except Exception:  # pragma: no cover
        import traceback
        q.put(traceback.format_exc())


def test_shared_cursor_across_processes():
    name = uuid.uuid4().hex
    total, n, boundary = 10_000, 37, 1000
    c = pg_scan.SharedCursor(name, nblocks=total, start=0, create=True)
    try:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_cursor_worker, args=(name, n, boundary, q)) for _ in range(4)]
        [p.start() for p in ps]
        parts = [q.get(timeout=120) for _ in ps]
        [p.join(timeout=60) for p in ps]
        claims = [x for p in parts for x in p]
        assert all(isinstance(p, list) for p in parts), parts
        cover = np.zeros(total, np.int32)
        for lo, k in claims:
            assert lo // boundary == (lo + k - 1) // boundary      # never crosses a segment
            cover[lo:lo + k] += 1
        assert (cover == 1).all()                                # every block exactly once
        cnt = c.counters()
        assert cnt["pages"] == total and cnt["tuples"] == total and cnt["chunks"] == len(claims)
        c.rescan()
        assert c.claim(5) == (0, 5)
    finally:
        c.close()
    assert not os.path.exists(c.path)


def test_plan_scan_decisions():
    cfg = pg_scan.ScanConfig()
    gib = 1 << 30
    small = pg_scan.plan_scan(1 << 20, 1000, 64 * gib, 8 * gib, cfg)
    assert small.path == "seqscan" and "threshold" in small.reason
    big = pg_scan.plan_scan(100 * gib, 10 ** 9, 64 * gib, 8 * gib, cfg, parallel_workers=4)
    assert big.path == "nvme_strom" and big.workers == 4 and big.cost < big.seqscan_cost
    assert "NVMEStrom" in big.explain()
    assert pg_scan.plan_scan(100 * gib, 10, 64 * gib, 8 * gib, cfg,
                             tablespace_ok=False).path == "seqscan"
    off = pg_scan.ScanConfig(enabled=False)
    assert pg_scan.plan_scan(100 * gib, 10, 64 * gib, 8 * gib, off).reason == "disabled"
    forced = pg_scan.ScanConfig(debug_no_threshold=True)
    assert pg_scan.plan_scan(1 << 20, 10, 64 * gib, 8 * gib, forced).path == "nvme_strom"


def test_heap_scan_pool_keyed_and_released(tmp_path, monkeypatch):
    """pooled participant resources are keyed by the configuration
    they were sized for, and released by close(), the context manager, or
    garbage collection of an unclosed scan object."""
    import gc
    from nvme_strom_amd.models import pg_scan
    from nvme_strom_amd.utils import pgpage
    data = pgpage.build_table(np.arange(300, dtype=np.int64), per_page=150, width=8)
    rel = pg_scan.Relation.write(str(tmp_path / "16384"), data, relseg_size=64)
    freed = []
    monkeypatch.setattr(pg_scan.HeapRelationScan, "_free", staticmethod(lambda rs: freed.append(rs)))
    cfg = pg_scan.ScanConfig(chunk_size=2 * 8192, buffer_size=8 * 8192)
    hs = pg_scan.HeapRelationScan(rel, cfg, "cpu")
    hs._release("A")
    assert hs._acquire() == "A" and freed == []          # same configuration: reused
    hs._release("A")
    hs.cfg = pg_scan.ScanConfig(chunk_size=4 * 8192, buffer_size=8 * 8192)
    monkeypatch.setattr(pg_scan, "HbmBuffer", lambda *a, **k: (_ for _ in ()).throw(RuntimeError("x")))
    with pytest.raises(RuntimeError):
        hs._acquire()                                     # mismatched entry freed first
    assert freed == ["A"]
    with pg_scan.HeapRelationScan(rel, cfg, "cpu") as h2:
        h2._release("B")
    assert freed == ["A", "B"]
    h3 = pg_scan.HeapRelationScan(rel, cfg, "cpu")
    h3._release("C")
    del h3
    gc.collect()
    assert freed == ["A", "B", "C"]


# ------------------------------------------------ HeapTupleSatisfiesMVCC parity
from nvme_strom_amd.utils.pgmvcc import (HEAP_COMBOCID, HEAP_XMAX_EXCL_LOCK, HEAP_XMAX_INVALID,  # noqa: E402
                                         HEAP_XMAX_IS_MULTI, HEAP_XMAX_LOCK_ONLY, HEAP_XMIN_COMMITTED,
                                         HEAP_XMIN_INVALID, MX_FOR_SHARE, MX_FOR_UPDATE, MX_UPDATE,
                                         MultiXact, SubTrans, XACT_ABORTED, XACT_COMMITTED,
                                         XACT_IN_PROGRESS, XACT_SUBCOMMITTED)

W = 1 << 32


def _hdr(xmin, xmax, mask, cid=0):
    return struct.pack("<IIIHHHHHB", xmin % W, xmax % W, cid, 0, 0, 0, 1, mask, 24)


def _both(xmin, xmax, mask, snap, clog, sub=None, mx=None, cid=0):
    nat = pgmvcc.native_visible(_hdr(xmin, xmax, mask, cid), snap, clog, sub, mx)
    mod = pgmvcc.model_visible(xmin % W, xmax % W, mask, cid, snap, clog, sub, mx)
    assert nat == mod, (xmin, xmax, hex(mask), cid, nat, mod)
    return nat


def test_mvcc_wraparound_snapshot():
    """A snapshot straddling the 2^32 wrap: ids compare modulo 2^32
    (TransactionIdPrecedes), so an xid just before the wrap precedes one
    just after it, and the commit-log window wraps with them."""
    base = W - 1000
    clog = CommitLog(4000, base=base)
    for x in range(base, base + 4000):
        clog.set(x % W, XACT_COMMITTED)
    snap = Snapshot(xmin=(W - 10) % W, xmax=20, xip=[W - 5, 7])
    old, running, after, late = W - 50, W - 5, 5, 30
    assert _both(old, 0, HEAP_XMAX_INVALID, snap, clog) is True      # before xmin
    assert _both(running, 0, HEAP_XMAX_INVALID, snap, clog) is False  # in xip
    assert _both(after, 0, HEAP_XMAX_INVALID, snap, clog) is True     # past the wrap, < xmax
    assert _both(7, 0, HEAP_XMAX_INVALID, snap, clog) is False        # in xip past the wrap
    assert _both(late, 0, HEAP_XMAX_INVALID, snap, clog) is False     # >= xmax
    # deleted by a committed xid before the wrap: gone; by one >= xmax: still there
    assert _both(old, W - 40, 0, snap, clog) is False
    assert _both(old, late, 0, snap, clog) is True
    # the old unsigned compare would call W - 50 >= xmax (20) and hide it
    assert pgmvcc.xid_precedes(W - 50, 20)


def test_mvcc_multixact_lockers_and_updaters():
    clog = CommitLog(2000)
    for x in range(3, 2000):
        clog.set(x, XACT_COMMITTED)
    clog.set(500, XACT_ABORTED)
    clog.set(600, XACT_IN_PROGRESS)
    mx = MultiXact(base=10)
    lockers = mx.add([(300, MX_FOR_SHARE), (301, MX_FOR_UPDATE)])
    upd_commit = mx.add([(300, MX_FOR_SHARE), (400, MX_UPDATE)])
    upd_abort = mx.add([(301, MX_FOR_SHARE), (500, MX_UPDATE)])
    upd_running = mx.add([(600, MX_UPDATE)])
    snap = Snapshot(xmin=650, xmax=700, xip=[])
    m = HEAP_XMIN_COMMITTED | HEAP_XMAX_IS_MULTI
    assert _both(100, lockers, m, snap, clog, mx=mx) is True          # lockers delete nothing
    assert _both(100, lockers, m | HEAP_XMAX_LOCK_ONLY, snap, clog, mx=mx) is True
    assert _both(100, upd_commit, m, snap, clog, mx=mx) is False      # committed update
    assert _both(100, upd_abort, m, snap, clog, mx=mx) is True        # aborted update
    snap2 = Snapshot(xmin=590, xmax=700, xip=[600])
    assert _both(100, upd_running, m, snap2, clog, mx=mx) is True     # updater still running
    # an xmax that is a multixact looked up in pg_xact would be nonsense: a
    # multi outside the window is undecided, not guessed
    assert _both(100, 999, m, snap, clog, mx=mx) is None
    # a pre-9.3 exclusive lock without IS_MULTI is a lock too
    assert _both(100, 400, HEAP_XMIN_COMMITTED | HEAP_XMAX_EXCL_LOCK, snap, clog) is True


def test_mvcc_subtransactions():
    """Sub-committed xids follow their parent (pg_subtrans); with an
    overflowed subxip the snapshot maps a subxid to its top-level xid."""
    clog = CommitLog(2000)
    sub = SubTrans(2000)
    clog.set(100, XACT_COMMITTED)
    clog.set(101, XACT_SUBCOMMITTED)
    sub.set(101, 100)                       # child of a committed parent
    clog.set(200, XACT_ABORTED)
    clog.set(201, XACT_SUBCOMMITTED)
    sub.set(201, 200)                       # child of an aborted parent
    clog.set(300, XACT_IN_PROGRESS)
    clog.set(301, XACT_SUBCOMMITTED)
    sub.set(301, 300)                       # child of a running parent
    snap = Snapshot(xmin=50, xmax=400, xip=[300], subxip=[301])
    mi = HEAP_XMAX_INVALID
    assert _both(101, 0, mi, snap, clog, sub) is True
    assert _both(201, 0, mi, snap, clog, sub) is False
    assert _both(301, 0, mi, snap, clog, sub) is False
    over = Snapshot(xmin=50, xmax=400, xip=[300], suboverflowed=True)
    assert _both(301, 0, mi, over, clog, sub) is False   # via its top-level xid
    assert _both(101, 0, mi, over, clog, sub) is True
    # without pg_subtrans a sub-committed xid cannot be decided
    assert _both(101, 0, mi, snap, clog, None) is None
    # deleted by a sub-committed child of a committed parent: gone
    assert _both(100, 101, 0, snap, clog, sub) is False
    assert _both(100, 201, 0, snap, clog, sub) is True


def test_mvcc_own_transaction():
    """The scanning transaction's own inserts / deletes by command id; a
    combo command id (inserted and deleted by it) is undecidable here."""
    clog = CommitLog(1000)
    for x in range(3, 1000):
        clog.set(x, XACT_COMMITTED)
    clog.set(700, XACT_IN_PROGRESS)
    clog.set(701, XACT_SUBCOMMITTED)
    snap = Snapshot(xmin=690, xmax=710, xip=[700], curxids=[700, 701], curcid=5)
    mi = HEAP_XMAX_INVALID
    assert _both(700, 0, mi, snap, clog, cid=3) is True        # inserted before the scan
    assert _both(701, 0, mi, snap, clog, cid=4) is True        # by its subtransaction
    assert _both(700, 0, mi, snap, clog, cid=5) is False       # inserted at / after it
    assert _both(100, 700, HEAP_XMIN_COMMITTED, snap, clog, cid=2) is False   # deleted before
    assert _both(100, 700, HEAP_XMIN_COMMITTED, snap, clog, cid=9) is True    # deleted after
    assert _both(700, 700, HEAP_COMBOCID, snap, clog, cid=1) is None
    # own insert, deleted by another (aborted) subtransaction not in curxids
    assert _both(700, 702, 0, snap, clog, cid=1) is True


def test_mvcc_native_equals_model_randomized():
    """Thousands of random headers — hint bits, multixacts, subtransactions,
    own xids, a window across the wrap — native == model, also through a
    page (removed + recheck line numbers)."""
    rng = np.random.default_rng(77)
    base = W - 3000
    n = 6000
    clog = CommitLog(n, base=base)
    sub = SubTrans(n, base=base)
    xs = [(base + i) % W for i in range(3, n)]
    for x in xs:
        st = int(rng.choice([XACT_COMMITTED] * 4 + [XACT_ABORTED, XACT_IN_PROGRESS,
                                                     XACT_SUBCOMMITTED]))
        clog.set(x, st)
        if st == XACT_SUBCOMMITTED or rng.random() < 0.2:
            sub.set(x, (x - int(rng.integers(1, 40))) % W)
    mx = MultiXact(base=W - 20)
    multis = [mx.add([(int(rng.choice(xs)), int(rng.integers(0, 6)))
                      for _ in range(int(rng.integers(1, 4)))]) for _ in range(60)]
    pick = lambda: int(rng.choice(xs))   # noqa: E731
    for trial in range(6):
        xmin = (base + int(rng.integers(1000, 3000))) % W
        xmax = (xmin + int(rng.integers(10, 2500))) % W
        xip = sorted({(xmin + int(rng.integers(0, 10))) % W for _ in range(5)})
        snap = Snapshot(xmin=xmin, xmax=xmax, xip=xip,
                        subxip=[pick() for _ in range(5)], suboverflowed=bool(trial % 2),
                        curxids=[pick(), pick()], curcid=int(rng.integers(0, 10)))
        for _ in range(500):
            ismulti = rng.random() < 0.2
            xmax_v = int(rng.choice(multis)) if ismulti else int(rng.choice([0] + xs))
            mask = int(rng.choice([0, HEAP_XMIN_COMMITTED, HEAP_XMIN_INVALID,
                                   HEAP_XMIN_COMMITTED | HEAP_XMIN_INVALID]))
            mask |= int(rng.choice([0, HEAP_XMAX_INVALID, 0x0400, HEAP_XMAX_LOCK_ONLY,
                                    HEAP_XMAX_EXCL_LOCK]))
            mask |= HEAP_XMAX_IS_MULTI if ismulti else 0
            mask |= HEAP_COMBOCID if rng.random() < 0.05 else 0
            xmin_v = int(rng.choice(snap.curxids)) if rng.random() < 0.1 else pick()
            _both(xmin_v, xmax_v, mask, snap, clog, sub, mx, cid=int(rng.integers(0, 10)))
        # a page: removed and recheck lists against the model
        cases = []
        for i in range(120):
            ismulti = rng.random() < 0.2
            xmax_v = int(rng.choice(multis)) if ismulti else int(rng.choice([0] + xs))
            mask = int(rng.choice([0, HEAP_XMIN_COMMITTED])) | (HEAP_XMAX_IS_MULTI if ismulti else 0)
            cases.append((i, pick(), xmax_v, mask))
        tuples = [pgpage.tuple_bytes(struct.pack("<q", i), infomask=m, xmin=a, xmax=b)
                  for i, a, b, m in cases]
        page = np.frombuffer(bytearray(pgpage.build_page(tuples, with_checksum=False)),
                             np.uint8).copy()
        rc = []
        removed = pgmvcc.apply_snapshot(page, snap, clog, subtrans=sub, multi=mx, recheck=rc)
        want = [pgmvcc.model_visible(a, b, m, 0, snap, clog, sub, mx) for i, a, b, m in cases]
        assert removed == sum(1 for w in want if w is False)
        assert rc == [i + 1 for i, w in enumerate(want) if w is None]


def test_read_check_pages_native_equals_per_tuple(tmp_path):
    """The host leg in native code (strom_pg_read_check_pages): pread of the
    blocks (runs across a segment's modulo), checksum verified then re-stamped
    after the edit, tuples removed and recheck flags — against the per-tuple
    native check and the Python model."""
    import mvccgen
    w = mvccgen.World(seed=3, n=3000)
    snap = w.snapshot(1)
    data, cases = w.pages(snap, 6, per_page=120)
    p = tmp_path / "rel"
    p.write_bytes(data)
    exp = w.expect(snap, cases, [True] * 6)
    for (keep, removed, rc), cs in zip(exp, cases):      # native == model
        for i, (a, b, m, c) in enumerate(cs):
            mod = pgmvcc.model_visible(a % W, b % W, m, c, snap, w.clog, w.sub, w.mx)
            assert (mod is False) == ((i + 1) not in keep)
    blocks = np.array([4, 5, 0, 1, 2], dtype=np.uint32)   # 6 blocks per "segment": 4,5 | 0,1,2
    stage = np.zeros(len(blocks) * 8192, np.uint8)
    fd = os.open(p, os.O_RDONLY)
    try:
        removed, rc = pgmvcc.read_check_pages(fd, blocks, stage, snap, w.clog, relseg_blocks=6,
                                              verify_checksum=True, subtrans=w.sub, multi=w.mx)
    finally:
        os.close(fd)
    assert removed == sum(exp[b][1] for b in blocks)
    assert rc.tolist() == [int(exp[b][2]) for b in blocks]
    for j, b in enumerate(blocks.tolist()):
        page = stage[j * 8192:(j + 1) * 8192].tobytes()
        items, status = pgpage.host_scan(page, 8192, verify_checksum=True, blkno_base=b)
        assert status == [0]                               # re-stamped checksum still valid
        assert [i & 0xFFFF for i in items] == exp[b][0]
