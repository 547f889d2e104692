"""Pipelines on CPU: SSD2RAM stream, PG scan planner pieces + CPU executor,
stream loader order restoration with page-cache chunks (emulated HBM)."""
import os

import struct

import numpy as np
import pytest

import nvme_strom_amd as S
from nvme_strom_amd.models import pg_scan
from nvme_strom_amd.models.ssd2ram_stream import ssd2ram_run
from nvme_strom_amd.utils import pgpage


def test_ssd2ram_stream_verified(strom, rand_file):
    path, data = rand_file(24 << 20)
    st = ssd2ram_run(path, nthreads=3, unit=1 << 20, buffer_sz=6 << 20, verify=True,
                     bind_numa=False)
    assert st.mismatches == 0
    assert st.nr_ssd + st.nr_ram == (24 << 20) // 8192
    assert st.bytes == 24 << 20


def test_stream_loader_restores_order_with_cached_chunks(strom, rand_file):
    import torch
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    path, data = rand_file(8 << 20, evict=False)           # fully cached
    ld = StreamLoader(path, segment_sz=2 << 20, nr_segments=4, chunk_sz=8192, device="cpu", depth=2)
    st = ld.run(0, 8 << 20)
    assert st.nr_ram > 0
    assert np.array_equal(ld.buf.tensor.numpy(), data)
    ld.close()


def test_planner_threshold_and_cost():
    cfg = pg_scan.ScanConfig()
    gib = 1 << 30
    thr = pg_scan.strom_threshold(64 * gib, 8 * gib)
    assert thr == (56 * gib) * 2 // 3 + 8 * gib
    assert not pg_scan.use_strom(thr - 1, 64 * gib, 8 * gib, cfg, True)
    assert pg_scan.use_strom(thr, 64 * gib, 8 * gib, cfg, True)
    assert not pg_scan.use_strom(thr, 64 * gib, 8 * gib, cfg, False)
    cfg.debug_no_threshold = True
    assert pg_scan.use_strom(1, 64 * gib, 8 * gib, cfg, True)
    assert pg_scan.scan_cost(1000, cfg, 2) < pg_scan.scan_cost(1000, cfg, 0)
    with pytest.raises(ValueError):
        pg_scan.ScanConfig(chunk_size=1000).validate()


def test_tablespace_cache(strom, tmp_path):
    c = pg_scan.TablespaceCache()
    assert c.can_use(str(tmp_path)) is True
    assert c.can_use(str(tmp_path / "missing")) is False
    c.invalidate()
    assert c.can_use(str(tmp_path)) is True


def test_parallel_cursor_boundaries():
    cur = pg_scan.ParallelCursor(100)
    got = []
    while True:
        lo, n = cur.claim(16, boundary=40)
        if not n:
            break
        got.append((lo, n))
        assert lo // 40 == (lo + n - 1) // 40
    assert sum(n for _, n in got) == 100


def test_cpu_scan_segments_and_filter(strom, tmp_path):
    vals = np.arange(2000, dtype=np.int64)
    data = pgpage.build_table(vals, per_page=100, width=8, invisible_every=10)   # 20 pages
    rel = pg_scan.Relation.write(str(tmp_path / "16384"), data, relseg_size=8)    # 3 segment files
    assert len(rel.segments) == 3 and rel.nblocks == 20
    cfg = pg_scan.ScanConfig(chunk_size=4 * 8192, buffer_size=8 * 8192, verify_checksum=True)
    for seg in rel.segments:
        fd = os.open(seg, os.O_RDONLY)
        S.api.evict_file(fd)
        os.close(fd)
    r = pg_scan.cpu_scan(rel, cfg, attr_off=0, attr_width=8, lo=100, hi=299)
    exp = [v for v in range(100, 300) if v % 10 != 0]
    assert r.ntuples == len(exp) and r.bad_pages == 0
    blocks = (r.items >> np.uint64(16)).astype(int)
    assert set(blocks.tolist()) == {1, 2}
    # per-scan counters (the reference's DSM stats) add up and are shown
    assert r.nr_ram + r.nr_ssd == 20 and r.chunks == 5   # segments of 8+8+4 blocks, 4 per chunk
    assert r.nr_ssd == 20 and r.nr_dma_submit >= 5 and r.nr_dma_blocks == 20 * 16
    text = r.explain()
    assert f"actual rows={len(exp)}" in text and "ssd2dev=" in text and "DMA: submits=" in text


def test_arrow_ipc_metadata(tmp_path):
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc as ipc
    from nvme_strom_amd.utils.arrow_ipc import read_metadata
    n = 10000
    a = np.arange(n, dtype=np.int64) * 3
    tbl = pa.table({"s": pa.array([str(i) for i in range(n)]), "a": a,
                    "f": pa.array(np.linspace(0, 1, n), type=pa.float32()),
                    "l": pa.array([[i, i + 1] for i in range(n)])})
    for comp in (None, "lz4"):
        path = str(tmp_path / f"m_{comp}.arrow")
        with ipc.new_file(path, tbl.schema, options=ipc.IpcWriteOptions(compression=comp)) as w:
            for k in range(4):
                w.write_batch(tbl.slice(k * 2500, 2500).to_batches()[0])
        m = read_metadata(path)
        # native header reader (csrc/engine/arrow_meta.cc) == the Python walk,
        # and == an in-memory source
        assert m == read_metadata(path, native=False)
        assert m == read_metadata(open(path, "rb").read())
        assert [c.name for c in m.schema] == ["s", "a", "f", "l"]
        assert [c.supported for c in m.schema] == [True, True, True, False]
        assert m.schema[2].numpy_dtype == "f4"
        assert len(m.batches) == 4 and all(b.length == 2500 for b in m.batches)
        assert m.batches[0].codec == (None if comp is None else "lz4_frame")
        if comp is None:
            raw = np.fromfile(path, dtype=np.uint8)
            for k, b in enumerate(m.batches):
                ref = b.columns[1].data
                vals = raw[ref.offset:ref.offset + 2500 * 8].view(np.int64)
                assert np.array_equal(vals, a[k * 2500:(k + 1) * 2500])


def test_arrow_headers_malformed(tmp_path):
    """A corrupted record-batch header is an error naming the batch, from
    the native reader and from the Python walk (never a wild read)."""
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc as ipc
    from nvme_strom_amd.utils.arrow_ipc import read_metadata
    tbl = pa.table({"a": np.arange(4000, dtype=np.int64)})
    path = str(tmp_path / "ok.arrow")
    with ipc.new_file(path, tbl.schema) as w:
        for k in range(4):
            w.write_batch(tbl.slice(k * 1000, 1000).to_batches()[0])
    m = read_metadata(path)
    raw = bytearray(open(path, "rb").read())
    hdr = m.batches[2].offset
    rng = np.random.default_rng(3)
    for trial in range(40):
        bad = bytearray(raw)
        # clobber the root offset / vtable region of batch 2's message
        pos = hdr + 8 + int(rng.integers(0, 24))
        bad[pos:pos + 4] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        p = str(tmp_path / f"bad{trial}.arrow")
        open(p, "wb").write(bad)
        for native in (True, False):
            try:
                got = read_metadata(p, native=native)
            except (ValueError, struct.error, IndexError, KeyError, UnicodeDecodeError):
                continue
            # an edit that still parses must leave the other batches intact
            assert got.batches[0] == m.batches[0] or not native


def test_arrow_headers_fuzz_asan(tmp_path):
    """20k random edits of a real header through the native parser built
    with ASan + UBSan (csrc/tests/arrow_meta_fuzz.cc)."""
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc as ipc
    import subprocess
    from nvme_strom_amd.utils.arrow_ipc import read_metadata
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "build/arrow_meta_fuzz"], cwd=root, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rng = np.random.default_rng(0)
    tbl = pa.table({"a": np.arange(4000, dtype=np.int64),
                    "x": pa.array(rng.random(4000), mask=rng.random(4000) < 0.1)})
    path = str(tmp_path / "f.arrow")
    with ipc.new_file(path, tbl.schema, options=ipc.IpcWriteOptions(compression="lz4")) as w:
        for k in range(4):
            w.write_batch(tbl.slice(k * 1000, 1000).to_batches()[0])
    b = read_metadata(path).batches[1]
    r = subprocess.run([os.path.join(root, "build", "arrow_meta_fuzz"), path, str(b.offset),
                        str(b.body_offset - b.offset), "20000"], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, TMPDIR=str(tmp_path)))
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "arrow_meta_fuzz:" in r.stdout and "rejected" in r.stdout


def test_cpu_scan_block_range_and_resumable(strom, tmp_path):
    """Block-range scans + checkpoint/resume: an interrupted ResumableScan
    continues at the first unscanned block and equals one full scan."""
    vals = np.arange(2000, dtype=np.int64)
    data = pgpage.build_table(vals, per_page=100, width=8, invisible_every=10)   # 20 pages
    rel = pg_scan.Relation.write(str(tmp_path / "16385"), data, relseg_size=8)
    cfg = pg_scan.ScanConfig(chunk_size=4 * 8192, buffer_size=8 * 8192, verify_checksum=True)
    pred = dict(attr_off=0, attr_width=8, lo=50, hi=1749)
    full = pg_scan.cpu_scan(rel, cfg, **pred)
    part = pg_scan.cpu_scan(rel, cfg, blocks=(5, 13), **pred)     # crosses a segment boundary
    blocks = set((part.items >> np.uint64(16)).astype(int).tolist())
    assert blocks == set(range(5, 13)) and part.pages == 8
    sel = (full.items >> np.uint64(16) >= 5) & (full.items >> np.uint64(16) < 13)
    assert np.array_equal(part.items, full.items[sel])
    with pytest.raises(ValueError):
        pg_scan.cpu_scan(rel, cfg, blocks=(7, 3), **pred)

    ck = str(tmp_path / "scan.ckpt.npz")
    scan = lambda b0, b1: pg_scan.cpu_scan(rel, cfg, blocks=(b0, b1), **pred)
    a = pg_scan.ResumableScan(scan, rel.nblocks, ck, step_blocks=3, key="16385:50-1749")
    assert a.run(max_steps=2) is None and a.next_block == 6       # "interrupted"
    b = pg_scan.ResumableScan(scan, rel.nblocks, ck, step_blocks=3, key="16385:50-1749")
    assert b.next_block == 6 and b.counters["pages"] == 6
    r = b.run()
    assert r is not None and np.array_equal(r.items, full.items)
    assert r.pages == 20 and r.nr_ram + r.nr_ssd == 20 and r.bad_pages == 0
    # a finished checkpoint reloads as done; a different key is refused
    c = pg_scan.ResumableScan(scan, rel.nblocks, ck, step_blocks=3, key="16385:50-1749")
    assert c.done and np.array_equal(c.run().items, full.items)
    with pytest.raises(ValueError):
        pg_scan.ResumableScan(scan, rel.nblocks, ck, step_blocks=3, key="other")
    # a different step size, or no key at all, is refused too
    with pytest.raises(ValueError):
        pg_scan.ResumableScan(scan, rel.nblocks, ck, step_blocks=4, key="16385:50-1749")
    with pytest.raises(ValueError):
        pg_scan.ResumableScan(scan, rel.nblocks, str(tmp_path / "x.npz"), step_blocks=3, key="")
    # per-range item files: each holds only its own range's rows
    names = sorted(c.ranges)
    assert len(names) == 7 and all(os.path.exists(tmp_path / n) for n in names)
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".tmp")]
    c.remove()
    assert not os.path.exists(ck) and not any(os.path.exists(tmp_path / n) for n in names)


def test_scan_key_tracks_relation_and_predicate(strom, tmp_path):
    data = pgpage.build_table(np.arange(300, dtype=np.int64), per_page=100, width=8)
    rel = pg_scan.Relation.write(str(tmp_path / "16390"), data)
    k1 = pg_scan.scan_key(rel, attr_off=0, lo=1, hi=5)
    assert k1 == pg_scan.scan_key(rel, attr_off=0, lo=1, hi=5)
    assert k1 != pg_scan.scan_key(rel, attr_off=0, lo=1, hi=6)
    assert k1 != pg_scan.scan_key(rel, pg_scan.ScanConfig(verify_checksum=True), attr_off=0, lo=1, hi=5)


def test_arrow_scan_plans_zstd_and_refuses_mixed(tmp_path):
    """ArrowScan's plan (no GPU needed) takes a pyarrow ZSTD file with the
    zstd decoder's codec and refuses a file mixing LZ4 and ZSTD batches."""
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc as ipc
    from nvme_strom_amd.models.arrow_scan import ArrowScan
    from nvme_strom_amd.ops import decompress as D
    tbl = pa.table({"a": np.arange(50_000, dtype=np.int64) * 7})
    path = str(tmp_path / "z.arrow")
    with ipc.new_file(path, tbl.schema, options=ipc.IpcWriteOptions(compression="zstd")) as w:
        for k in range(4):
            w.write_batch(tbl.slice(k * 12_500, 12_500).to_batches()[0])
    sc = ArrowScan(path, "cpu")
    batches, dtypes, rows = sc._plan(["a"])
    assert sc._codec == D.ARROW_ZSTD and rows == 50_000 and len(batches) == 4
    assert all(d.compressed for b in batches for d, *_ in b.cols)
    mixed = str(tmp_path / "m.arrow")
    with ipc.new_file(mixed, tbl.schema, options=ipc.IpcWriteOptions(compression="zstd")) as w:
        w.write_batch(tbl.slice(0, 100).to_batches()[0])
    # pyarrow writes one codec per file: the mixed case is built in the metadata
    sc2 = ArrowScan(mixed, "cpu")
    sc2.meta.codecs = ["zstd", "lz4_frame"]
    with pytest.raises(NotImplementedError):
        sc2._plan(["a"])
