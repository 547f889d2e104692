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
    """Independent model of the MVCC rules the native check applies."""
    def st(x):
        return clog.status(x)

    def sees(x):
        return snap.sees(x)
    frozen = (mask & (XMIN_C | XMIN_I)) == (XMIN_C | XMIN_I)
    if not frozen:
        if mask & XMIN_I:
            return False
        if not (mask & XMIN_C or st(xmin) == 1) or not sees(xmin):
            return False
    if mask & XMAX_I or xmax == 0 or mask & 0x0080:
        return True
    deleted = bool(mask & XMAX_C) or st(xmax) == 1
    return not (deleted and sees(xmax))


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
