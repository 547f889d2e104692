"""GPU pipelines: PG heap relation scan vs the CPU executor, Arrow IPC scan vs
pyarrow, multi-window fan-out at world size 1."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nvme_strom_amd as S
    S.configure(gpu_emulation=0)
    return S


def test_pg_relation_scan_gpu_vs_cpu(S, tmp_path):
    from nvme_strom_amd.models import pg_scan
    from nvme_strom_amd.utils import pgpage
    rng = np.random.default_rng(0)
    vals = rng.integers(-5000, 5000, 30000).astype(np.int64)
    data = pgpage.build_table(vals, per_page=150, width=8, invisible_every=9)
    rel = pg_scan.Relation.write(str(tmp_path / "24576"), data, relseg_size=64)
    # warm a few blocks so some chunks take the page-cache (RAM) path
    fd = os.open(rel.segments[1], os.O_RDONLY)
    os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_RANDOM)
    for b in (3, 4, 5, 40):
        os.pread(fd, 8192, b * 8192)
    os.close(fd)
    cfg = pg_scan.ScanConfig(chunk_size=16 * 8192, buffer_size=64 * 8192, verify_checksum=True)
    for workers in (1, 3):
        with pg_scan.HeapRelationScan(rel, cfg, "cuda", attr_off=0, attr_width=8, lo=-100,
                                      hi=2500) as hs:
            g = hs.run(workers)
        c = pg_scan.cpu_scan(rel, cfg, attr_off=0, attr_width=8, lo=-100, hi=2500)
        assert np.array_equal(g.items, c.items)
        assert g.bad_pages == 0 and g.pages == rel.nblocks


def test_pg_relation_scan_resumable_gpu(S, tmp_path):
    """GPU block-range scans under ResumableScan, interrupted and resumed,
    equal one full CPU scan."""
    from nvme_strom_amd.models import pg_scan
    from nvme_strom_amd.utils import pgpage
    vals = np.random.default_rng(5).integers(-5000, 5000, 24000).astype(np.int64)
    data = pgpage.build_table(vals, per_page=150, width=8, invisible_every=7)   # 160 pages
    rel = pg_scan.Relation.write(str(tmp_path / "24577"), data, relseg_size=64)
    cfg = pg_scan.ScanConfig(chunk_size=16 * 8192, buffer_size=64 * 8192, verify_checksum=True)
    pred = dict(attr_off=0, attr_width=8, lo=-1000, hi=3000)
    full = pg_scan.cpu_scan(rel, cfg, **pred)
    with pg_scan.HeapRelationScan(rel, cfg, "cuda", **pred) as g:
        ck = str(tmp_path / "gpu.ckpt.npz")
        scan = lambda b0, b1: g.run(2, blocks=(b0, b1))
        a = pg_scan.ResumableScan(scan, rel.nblocks, ck, step_blocks=50, key="24577")
        assert a.run(max_steps=1) is None and a.next_block == 50
        r = pg_scan.ResumableScan(scan, rel.nblocks, ck, step_blocks=50, key="24577").run()
    assert np.array_equal(r.items, full.items) and r.pages == rel.nblocks and r.bad_pages == 0


@pytest.mark.parametrize("codecs", [("lz4", None), ("zstd",)])
def test_arrow_scan(S, tmp_path, codecs):
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc as ipc
    from nvme_strom_amd.models.arrow_scan import ArrowScan
    rng = np.random.default_rng(3)
    n, nb = 250_000, 5
    a = rng.integers(-10**6, 10**6, n * nb)
    b = rng.random(n * nb)
    mask = rng.random(n * nb) < 0.05
    tbl = pa.table({"a": pa.array(a, type=pa.int64()),
                    "b": pa.array(b, type=pa.float64(), mask=mask),
                    "s": pa.array([str(x % 100) for x in range(n * nb)])})
    path = str(tmp_path / "t.arrow")
    for comp in codecs:
        with ipc.new_file(path, tbl.schema, options=ipc.IpcWriteOptions(compression=comp)) as w:
            for k in range(nb):
                w.write_batch(tbl.slice(k * n, n).to_batches()[0])
        sc = ArrowScan(path, "cuda")
        out = sc.filter("a", -1000, 5000)
        ref = np.nonzero((a >= -1000) & (a <= 5000))[0]
        assert out.selected == len(ref)
        assert np.array_equal(out.indices.cpu().numpy(), ref)
        out = sc.filter("b", 0.25, 0.5)
        ref = np.nonzero((b >= 0.25) & (b <= 0.5) & ~mask)[0]
        assert np.array_equal(out.indices.cpu().numpy(), ref)
        # a qualifier list over two columns (each read and decoded once,
        # bitmaps ANDed on the device) + a projected third column
        sel = (a >= -500_000) & (a <= 200_000) & (b >= 0.1) & (b <= 0.6) & ~mask
        ref = np.nonzero(sel)[0]
        out = sc.scan_where([("a", -500_000, 200_000), ("b", 0.1, 0.6)], project="a")
        assert out.selected == len(ref)
        assert np.array_equal(out.indices.cpu().numpy(), ref)
        assert np.array_equal(out.values.cpu().numpy(), a[ref])
        # projecting a column with nulls returns its validity too
        out = sc.scan_where([("a", -500_000, 200_000)], project="b")
        ref = np.nonzero((a >= -500_000) & (a <= 200_000))[0]
        assert np.array_equal(out.indices.cpu().numpy(), ref)
        v = out.valid.cpu().numpy().astype(bool)
        assert np.array_equal(v, ~mask[ref])
        assert np.array_equal(out.values.cpu().numpy()[v], b[ref][v])
        sc.close()
        # record-batch ranges (the multi-rank split): ids stay file-global
        sc = ArrowScan(path, "cuda")
        parts = [sc.scan_where([("a", -1000, 5000)], batches=r).indices.cpu().numpy()
                 for r in ((0, 2), (2, 2), (2, 5))]
        ref = np.nonzero((a >= -1000) & (a <= 5000))[0]
        assert np.array_equal(np.concatenate(parts), ref)
        sc.close()


def test_arrow_scan_bar_refused_after_cold_scan(S, tmp_path):
    """a cold one-column scan (no page-cache chunks, so the reader
    never learns the BAR is refused), then a warm two-column scan_where whose
    groups are larger, with the large-BAR mapping off: the page-cache chunks
    go through a per-slot write-back buffer sized for the larger groups."""
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc as ipc
    from nvme_strom_amd.models.arrow_scan import ArrowScan
    rng = np.random.default_rng(7)
    n, nb = 200_000, 4
    a = rng.integers(-10**6, 10**6, n * nb)
    b = rng.integers(-10**6, 10**6, n * nb)
    tbl = pa.table({"a": pa.array(a, type=pa.int64()), "b": pa.array(b, type=pa.int64())})
    path = str(tmp_path / "w.arrow")
    with ipc.new_file(path, tbl.schema) as w:
        for k in range(nb):
            w.write_batch(tbl.slice(k * n, n).to_batches()[0])
    S.configure(bar_map=0)
    try:
        fd = os.open(path, os.O_RDONLY)
        S.evict_file(fd)
        os.close(fd)
        sc = ArrowScan(path, "cuda")
        out = sc.filter("a", -1000, 5000)
        assert np.array_equal(out.indices.cpu().numpy(), np.nonzero((a >= -1000) & (a <= 5000))[0])
        with open(path, "rb") as f:     # now every chunk is in the page cache
            f.read()
        sel = (a >= -500_000) & (a <= 200_000) & (b >= 0) & (b <= 700_000)
        out = sc.scan_where([("a", -500_000, 200_000), ("b", 0, 700_000)], project="b")
        ref = np.nonzero(sel)[0]
        assert np.array_equal(out.indices.cpu().numpy(), ref)
        assert np.array_equal(out.values.cpu().numpy(), b[ref])
        sc.close()
    finally:
        S.configure(bar_map=1)


def test_distributed_scan_two_ranks_one_gpu(tmp_path):
    """parallel/scan.py end to end on the GPU: 2 ranks (gloo, both on the
    box's one GPU, collectives staged via host memory) each scan their share
    of the record batches; rank 0 verifies the combined ids and projected
    values against numpy."""
    pytest.importorskip("pyarrow")
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29547", "-m",
           "nvme_strom_amd.tools.dist_scan_bench", "--rows", str(1 << 21), "--batch-rows",
           str(1 << 14), "--dir", str(tmp_path), "--reps", "1", "--backend", "gloo"]
    p = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["world"] == 2 and out["verified"] is True
    assert sum(out["per_rank_selected"]) == out["selected"] > 0
    assert out["ranges"][0][0] == 0 and out["ranges"][0][1] == out["ranges"][1][0]
    assert all(b > 0 for b in out["bytes_read_per_rank"])


def test_distributed_heap_scan_two_ranks_one_gpu(tmp_path):
    """DistributedHeapScan on the GPU: 2 ranks (gloo, one GPU) claim chunks
    of one relation from a shared cursor; rank 0 checks the combined item
    pointers against the CPU executor."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29549", "-m",
           "nvme_strom_amd.tools.dist_scan_bench", "--kind", "pg", "--pg-mib", "64",
           "--dir", str(tmp_path), "--reps", "1", "--backend", "gloo"]
    p = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["world"] == 2 and out["verified"] is True
    assert sum(out["per_rank_items"]) == out["items"] > 0
    assert out["pages_total"] == out["relation_bytes"] // 8192


def test_sharded_loader_single_rank(S, tmp_path):
    from nvme_strom_amd.parallel import ShardedLoader
    data = np.random.default_rng(1).integers(0, 256, 16 << 20, dtype=np.uint8)
    p = str(tmp_path / "s.bin")
    data.tofile(p)
    ld = ShardedLoader(p, 4 << 20, torch.device("cuda"), segment_sz=1 << 20, depth=3)
    for i in range(5):
        ld.step(i)
        ld.flush()
        exp = data[(i % 4) * (4 << 20):][:4 << 20]
        assert np.array_equal(ld.current(i).cpu().numpy(), exp)
    ld.close()


def test_heap_scan_vm_routing_matches_cpu(S, tmp_path):
    """MVCC mode on the GPU: all-visible blocks DMA'd unchecked, the others
    snapshot-checked on the host and copied behind them in HBM; the rows
    equal the reference-shaped CPU path's."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_pg_mvcc_cpu import _mvcc_relation
    from nvme_strom_amd.models import pg_scan
    rel, snap, clog, want, nchecked = _mvcc_relation(tmp_path, nblocks=40)
    cfg = pg_scan.ScanConfig(chunk_size=6 * 8192, buffer_size=18 * 8192, snapshot=snap,
                             clog=clog, verify_checksum=True)
    with pg_scan.HeapRelationScan(rel, cfg, "cuda") as hs:
        g = hs.run(workers=2)
    assert set(g.items.tolist()) == want
    assert g.nr_checked == nchecked and g.bad_pages == 0
    c = pg_scan.cpu_scan(rel, cfg)
    assert np.array_equal(g.items, c.items)


@pytest.mark.parametrize("codec", [None, "lz4", "zstd"])
def test_arrow_scan_predicate_kinds(S, tmp_path, codec):
    """Every predicate kind on every column kind (tests/arrowgen.py) through
    the GPU qualifier kernel: row ids == pc.filter of pyarrow.compute's mask,
    and == the host twin; qualifier lists (CNF with OR clauses) with a
    timestamp / dictionary projection."""
    pytest.importorskip("pyarrow")
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from arrowgen import cases, cnf_cases, expected_ids, table, write
    from nvme_strom_amd.models.arrow_scan import ArrowScan
    tbl = table(6000, seed=11)
    path = str(tmp_path / f"p_{codec}.arrow")
    write(path, tbl, codec, batch_rows=1000)
    sc = ArrowScan(path, "cuda", chunk_sz=64 << 10, slot_bytes=1 << 20)
    try:
        bad = []
        for label, pred, ref in cases():
            got = sc.scan_where([pred]).indices.cpu().numpy()
            want = expected_ids(tbl, ref)
            if not np.array_equal(got, want):
                bad.append((label, len(got), len(want)))
        assert not bad, bad
        for label, quals, ref in cnf_cases():
            out = sc.scan_where(quals, project="ts")
            want = expected_ids(tbl, ref)
            assert np.array_equal(out.indices.cpu().numpy(), want), label
            ts = tbl.column("ts").combine_chunks()
            ok = np.asarray(ts.is_valid())[want]
            assert np.array_equal(out.valid.cpu().numpy().astype(bool), ok)
            ref_v = np.asarray(ts.cast("int64").fill_null(0))[want]
            assert np.array_equal(out.values.cpu().numpy()[ok], ref_v[ok])
            assert out.column.kind == "timestamp" and out.column.unit == "us"
        from nvme_strom_amd.ops.colpred import P
        out = sc.scan_where([P("i8") > 60], project="dict")
        d = tbl.column("dict").combine_chunks()
        ids = out.indices.cpu().numpy()
        ok = np.asarray(d.is_valid())[ids]
        assert np.array_equal(out.values.cpu().numpy()[ok],
                              np.asarray(d.indices.fill_null(0))[ids][ok])
        offs, chars = out.dictionary[0]
        assert [chars[offs[i]:offs[i + 1]].tobytes().decode() for i in range(len(offs) - 1)] == \
            d.dictionary.to_pylist()
        # utf8 / large utf8 / binary projections: characters + offsets
        for pc_name in ("s", "ls", "bin"):
            out = sc.scan_where([P("i8") > 30], project=pc_name)
            ids = out.indices.cpu().numpy()
            col = tbl.column(pc_name).combine_chunks()
            offs = out.offsets.cpu().numpy()
            chars = out.values.cpu().numpy().tobytes()
            ok = np.asarray(col.is_valid())[ids]
            if out.valid is not None:
                assert np.array_equal(out.valid.cpu().numpy().astype(bool), ok)
            got = [chars[offs[i]:offs[i + 1]] for i in range(len(ids))]
            want = [col[int(r)].as_py() for r in ids]
            want = [w.encode() if isinstance(w, str) else w for w in want]
            assert all(g == w for g, w, v in zip(got, want, ok) if v), pc_name
        # decimal128 projection: (lo, hi) words of the scaled integer
        out = sc.scan_where([P("i8") > 30], project="dec")
        ids = out.indices.cpu().numpy()
        w = out.values.cpu().numpy().astype(np.uint64)
        got = [int(lo) | (int(hi) << 64) for lo, hi in w]
        got = [g - (1 << 128) if g >> 127 else g for g in got]
        dcol = tbl.column("dec").combine_chunks()
        ok = np.asarray(dcol.is_valid())[ids]
        want = [int(dcol[int(r)].as_py().scaleb(4)) if v else None for r, v in zip(ids, ok)]
        assert all(g == x for g, x, v in zip(got, want, ok) if v)
        host = sc.host_scan_where([P("s").startswith("ap"), P("u32") < 1 << 31])
        assert np.array_equal(sc.scan_where([P("s").startswith("ap"), P("u32") < 1 << 31])
                              .indices.cpu().numpy(), host.indices)
    finally:
        sc.close()
