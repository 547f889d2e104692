"""Snapshot visibility on the GPU (heapscan.hip mvcc_visible):
HeapTupleSatisfiesMVCC's rules run by the scan kernel for every tuple of a
page the visibility map does not call all-visible, equal to the native host
check (strom_pg_tuple_visible, itself held against the Python model in
tests/test_pg_mvcc_cpu.py) on randomized fixtures — xids across the 2^32
wrap, sub-committed xids and overflowed snapshots, multixact lockers and
updaters, the scanning transaction's own xids and command ids, combo cids
(undecidable: kept, page flagged for the host recheck)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import mvccgen  # noqa: E402
from nvme_strom_amd.utils import pgmvcc  # noqa: E402


@pytest.fixture(scope="module")
def world():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return mvccgen.World(seed=77, n=6000)


def _check(r, exp, npages):
    items = r.sorted_items()
    got = [[] for _ in range(npages)]
    for it in items.tolist():
        got[it >> 16].append(it & 0xFFFF)
    assert got == [e[0] for e in exp]
    assert r.removed == sum(e[1] for e in exp)
    status = r.page_status.cpu().numpy()
    assert [bool(s & 8) for s in status.tolist()] == [e[2] for e in exp]


@pytest.mark.parametrize("bitmap", [True, False], ids=["bitmap", "search"])
@pytest.mark.parametrize("trial", range(6))
def test_device_mvcc_equals_native_randomized(world, trial, bitmap, monkeypatch):
    """Both XidInMVCCSnapshot forms on the device: the running-xid bitmap
    over [xmin, xmax) and the sorted-list binary search (snapshots too wide
    for a bitmap)."""
    from nvme_strom_amd.ops import heapscan as H
    if not bitmap:
        monkeypatch.setattr(H.DeviceMvcc, "RUNNING_MAX_BITS", 0)
    snap = world.snapshot(trial)
    npages = 12
    data, cases = world.pages(snap, npages, per_page=200, all_visible_every=5)
    pages = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    dm = H.DeviceMvcc(snap, world.clog, world.sub, world.mx)
    assert (dm.running is not None) == bitmap
    # PD_ALL_VISIBLE pages (0, 5, 10) are never checked
    exp = world.expect(snap, cases, [p % 5 != 0 for p in range(npages)])
    r = H.heap_scan(pages, verify_checksum=True, mvcc=dm)
    _check(r, exp, npages)
    # the VM's verdict per page: flag 0 = all-visible, taken unchecked
    flags = np.array([p % 3 != 0 for p in range(npages)], np.uint8)
    exp2 = world.expect(snap, cases, [bool(f) and p % 5 != 0 for p, f in enumerate(flags)])
    r2 = H.heap_scan(pages, mvcc=dm, mvcc_pages=flags)
    _check(r2, exp2, npages)


def test_device_mvcc_with_quals(world):
    """The snapshot check composed with a qualifier list (fixed AND list and
    program mode): a tuple needs both; undecided visibility keeps the tuple
    for the quals and flags its page."""
    from nvme_strom_amd.ops import heapscan as H
    from nvme_strom_amd.utils import pgtuple as T
    snap = world.snapshot(3)
    npages = 8
    data, cases = world.pages(snap, npages, per_page=150)
    pages = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    desc = T.TupleDesc.of([("v", "int8")])
    dm = H.DeviceMvcc(snap, world.clog, world.sub, world.mx)
    exp = world.expect(snap, cases, [True] * npages)
    for program in (False, True):
        r = H.heap_scan2(pages, desc, [T.Qual("v", "between", (0, 10 ** 9))], mvcc=dm,
                         program=program)
        _check(r, exp, npages)
        qs = [T.Qual("v", "between", (2000, 4999))]        # pages 2..4 by value
        r = H.heap_scan2(pages, desc, qs, mvcc=dm, program=program)
        want = [e[0] if 2 <= p <= 4 else [] for p, e in enumerate(exp)]
        items = r.sorted_items().tolist()
        got = [[i & 0xFFFF for i in items if i >> 16 == p] for p in range(npages)]
        assert got == want
        st = r.page_status.cpu().numpy().tolist()
        assert [bool(s & 8) for s in st] == [e[2] for e in exp]


def test_device_mvcc_directed_cases():
    """The directed cases of the host tests, through the kernel: wrap,
    multixact, subtransactions, own transaction and combo cid."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import struct
    from nvme_strom_amd.ops import heapscan as H
    from nvme_strom_amd.utils import pgpage
    from nvme_strom_amd.utils.pgmvcc import (HEAP_COMBOCID, HEAP_XMAX_INVALID, HEAP_XMIN_COMMITTED,
                                             CommitLog, Snapshot, SubTrans, XACT_ABORTED,
                                             XACT_COMMITTED, XACT_IN_PROGRESS, XACT_SUBCOMMITTED)
    W = 1 << 32
    clog = CommitLog(8000, base=W - 1000)
    sub = SubTrans(8000, base=W - 1000)
    for x in range(W - 1000, W + 7000):
        clog.set(x % W, XACT_COMMITTED)
    clog.set(200, XACT_ABORTED)
    clog.set(201, XACT_SUBCOMMITTED)
    sub.set(201, 200)
    clog.set(101, XACT_SUBCOMMITTED)
    sub.set(101, 100)
    clog.set(700, XACT_IN_PROGRESS)
    snap = Snapshot(xmin=(W - 10) % W, xmax=800, xip=[W - 5, 7, 700], curxids=[700], curcid=5)
    cases = [  # (xmin, xmax, mask, cid, want)
        (W - 50, 0, HEAP_XMAX_INVALID, 0, True),      # before xmin
        (W - 5, 0, HEAP_XMAX_INVALID, 0, False),      # running, before the wrap
        (5, 0, HEAP_XMAX_INVALID, 0, True),           # past the wrap, committed
        (7, 0, HEAP_XMAX_INVALID, 0, False),          # running, past the wrap
        (900, 0, HEAP_XMAX_INVALID, 0, False),        # >= xmax
        (W - 50, W - 40, 0, 0, False),                # deleted before the snapshot
        (101, 0, HEAP_XMAX_INVALID, 0, True),         # child of a committed parent
        (201, 0, HEAP_XMAX_INVALID, 0, False),        # child of an aborted parent
        (700, 0, HEAP_XMAX_INVALID, 3, True),         # own insert before the scan
        (700, 0, HEAP_XMAX_INVALID, 5, False),        # own insert at the scan's cid
        (100, 700, HEAP_XMIN_COMMITTED, 2, False),    # own delete before
        (100, 700, HEAP_XMIN_COMMITTED, 9, True),     # own delete after
        (700, 700, HEAP_COMBOCID, 1, None),           # combo cid: undecided
    ]
    tuples = [mvccgen.tuple_of(a, b, m, c, struct.pack("<q", i))
              for i, (a, b, m, c, _) in enumerate(cases)]
    page = pgpage.build_page(tuples, blkno=0)
    for a, b, m, c, want in cases:
        assert pgmvcc.native_visible(mvccgen.header(a, b, m, c), snap, clog, sub) is want
    pages = torch.frombuffer(bytearray(page), dtype=torch.uint8).cuda()
    r = H.heap_scan(pages, verify_checksum=True, mvcc=H.DeviceMvcc(snap, clog, sub))
    assert [i & 0xFFFF for i in r.sorted_items().tolist()] == \
        [i + 1 for i, cs in enumerate(cases) if cs[4] is not False]
    assert r.removed == sum(1 for cs in cases if cs[4] is False)
    assert int(r.page_status[0].item()) & 8
    assert r.recheck == 1


@pytest.mark.parametrize("device_mvcc", [True, False])
def test_relation_scan_snapshot_equals_cpu(tmp_path, device_mvcc):
    """HeapRelationScan with a snapshot — VM-routed, device check (default)
    or the host leg — equals cpu_scan: items, tuples removed, blocks checked,
    recheck blocks; with 1 and 3 participants and a qualifier list."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nvme_strom_amd as S
    from nvme_strom_amd.models import pg_scan
    from nvme_strom_amd.utils import pgtuple as T
    S.configure(gpu_emulation=0)
    w = mvccgen.World(seed=5, n=4000)
    snap = w.snapshot(1)
    nb = 40
    data, cases = w.pages(snap, nb, per_page=150, all_visible_every=7)
    av = [b % 4 == 0 for b in range(nb)]                  # VM bits (PD flag on 0, 7, 14, ...)
    rel = pg_scan.Relation.write(str(tmp_path / "30001"), data, relseg_size=16, all_visible=av)
    cfg = pg_scan.ScanConfig(chunk_size=6 * 8192, buffer_size=24 * 8192, verify_checksum=True,
                             snapshot=snap, clog=w.clog, subtrans=w.sub, multixact=w.mx,
                             mvcc_device=device_mvcc)
    c = pg_scan.cpu_scan(rel, cfg)
    exp = w.expect(snap, cases, [not av[b] and b % 7 != 0 for b in range(nb)])
    assert c.items.tolist() == [(b << 16) | i for b in range(nb) for i in exp[b][0]]
    assert c.removed == sum(e[1] for e in exp)
    for workers in (1, 3):
        with pg_scan.HeapRelationScan(rel, cfg, "cuda") as hs:
            g = hs.run(workers)
        assert np.array_equal(g.items, c.items)
        assert g.removed == c.removed and g.nr_checked == c.nr_checked
        assert sorted(g.recheck_blocks) == c.recheck_blocks
        assert g.bad_pages == 0
    desc = T.TupleDesc.of([("v", "int8")])
    qs = [T.Qual("v", "between", (3000, 20999))]
    cq = pg_scan.cpu_scan(rel, cfg, desc=desc, quals=qs, project="v")
    with pg_scan.HeapRelationScan(rel, cfg, "cuda", desc=desc, quals=qs, project="v") as hs:
        gq = hs.run(2)
    assert np.array_equal(gq.items, cq.items) and len(gq.items)
    assert np.array_equal(gq.values, cq.values)
