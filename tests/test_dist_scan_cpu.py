"""Multi-rank scans (parallel/scan.py) on CPU over gloo with 3 ranks: the
Arrow batch partition and combine step, and the PostgreSQL heap scan whose
ranks share one cross-process block cursor.

The GPU scan itself runs in tests/test_gpu_models.py; here each rank's
ArrowScan is replaced by a numpy scan of the same record-batch range of a
real pyarrow file, so what is tested is everything around it: ranges
covering the file exactly once, balanced by stored bytes, per-rank counts,
the padded variable-length all-gather, file order, projected values and
their validity (a rank without nulls must still join the validity gather).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nvme_strom_amd.parallel.scan import partition


def test_partition_exact_cover_and_balance():
    rng = np.random.default_rng(0)
    for n, parts in ((0, 3), (1, 4), (5, 5), (7, 3), (100, 8), (1000, 7)):
        w = rng.integers(1, 1000, n).astype(float)
        r = partition(w, parts)
        assert len(r) == parts
        assert r[0][0] == 0 and r[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))      # contiguous
        assert all(lo <= hi for lo, hi in r)
        if n >= 10 * parts:
            loads = [w[lo:hi].sum() for lo, hi in r]
            assert max(loads) <= w.sum() / parts + w.max() + 1e-9
    assert partition(np.zeros(6), 3) == [(0, 2), (2, 4), (4, 6)]
    assert partition(np.ones(4), 1) == [(0, 4)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _NumpyScan:
    """Stand-in for ArrowScan on CPU: same metadata, numpy evaluation of
    the batch range."""

    def __init__(self, path, device, **kw):
        import pyarrow as pa
        import pyarrow.ipc as ipc
        from nvme_strom_amd.utils.arrow_ipc import read_metadata
        self.meta = read_metadata(path)
        with pa.memory_map(path) as src:
            self.tbl = ipc.open_file(src).read_all()

    def scan_where(self, quals, project=None, batches=None):
        import torch
        from nvme_strom_amd.models.arrow_scan import ScanOut
        rows = self.meta.rows
        base = np.concatenate([[0], np.cumsum(rows)])
        lo, hi = base[batches[0]], base[batches[1]]
        m = np.ones(hi - lo, dtype=bool)
        for name, a, b in quals:
            c = self.tbl.column(name).combine_chunks().slice(lo, hi - lo)
            v = c.to_numpy(zero_copy_only=False)
            ok = ~np.asarray(c.is_null()) if c.null_count else np.ones(len(v), bool)
            m &= ok & (v >= a) & (v <= b)
        idx = np.flatnonzero(m) + lo
        vals = valid = None
        if project:
            c = self.tbl.column(project).combine_chunks()
            pv = c.to_numpy(zero_copy_only=False)[idx]
            vals = torch.from_numpy(np.nan_to_num(pv).copy())
            if c.null_count:
                valid = torch.from_numpy((~np.asarray(c.is_null())[idx]).astype(np.uint8))
        return ScanOut(int(hi - lo), len(idx), torch.from_numpy(idx.astype(np.int64)), {},
                       values=vals, valid=valid)

    def close(self):
        pass


def _worker(rank, world, port, path, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        import nvme_strom_amd.parallel.scan as PS
        PS.ArrowScan = _NumpyScan
        dist.init_process_group("gloo")
        ds = PS.DistributedArrowScan(path, torch.device("cpu"))
        a = ds.scan_where([("val", 100, 599), ("x", 0.2, 0.8)], project="x")
        b = ds.scan_where([("val", 0, 999)], project="id", gather="none")
        q.put((rank, dict(idx=a.indices.numpy(), vals=a.values.numpy(),
                          valid=None if a.valid is None else a.valid.numpy(),
                          counts=a.per_rank, ranges=a.ranges, mine=b.indices.numpy(),
                          mine_vals=b.values.numpy())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_distributed_scan_combine_3_ranks(tmp_path):
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc as ipc
    rng = np.random.default_rng(5)
    path = str(tmp_path / "d.arrow")
    schema = pa.schema([("id", pa.int64()), ("val", pa.int64()), ("x", pa.float64())])
    ids, vals, xs, nulls = [], [], [], []
    with ipc.new_file(path, schema, options=ipc.IpcWriteOptions(compression="lz4")) as w:
        base = 0
        for k in range(11):                            # uneven batch sizes
            n = int(rng.integers(50, 400))
            i = np.arange(base, base + n, dtype=np.int64)
            v = rng.integers(0, 1000, n, dtype=np.int64)
            x = rng.random(n)
            # nulls only in the first batches: some ranks have none
            msk = (rng.random(n) < 0.2) if k < 3 else np.zeros(n, bool)
            w.write_batch(pa.record_batch([pa.array(i), pa.array(v), pa.array(x, mask=msk)],
                                          schema=schema))
            ids.append(i), vals.append(v), xs.append(x), nulls.append(msk)
            base += n
    ids, vals, xs, nulls = map(np.concatenate, (ids, vals, xs, nulls))
    want = np.flatnonzero((vals >= 100) & (vals <= 599) & ~nulls & (xs >= 0.2) & (xs <= 0.8))
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r], dict), res[r]
    rngs = res[0]["ranges"]
    assert rngs[0][0] == 0 and rngs[-1][1] == 11 and all(a[1] == b[0] for a, b in zip(rngs, rngs[1:]))
    mine_all = []
    for r in range(world):
        d = res[r]
        assert d["ranges"] == rngs
        assert np.array_equal(d["idx"], want), r                 # every rank: full result
        assert np.allclose(d["vals"], xs[want])
        assert d["valid"] is not None and (d["valid"] == 1).all()  # selected rows are non-null
        assert sum(d["counts"]) == len(want)
        mine_all.append(d["mine"])
        assert np.array_equal(d["mine_vals"], d["mine"])         # id projected = row id
    assert np.array_equal(np.concatenate(mine_all), np.arange(len(ids)))   # sharded: file order


class _CpuHeapScan:
    """Stand-in for HeapRelationScan on CPU: claims chunks from the given
    cursor like the GPU participants and scans each with cpu_scan."""

    def __init__(self, rel, cfg, device, **pred):
        self.rel, self.cfg, self.pred = rel, cfg, pred

    def run(self, workers=1, blocks=None, cursor=None):
        from nvme_strom_amd.models import pg_scan
        parts, pages = [], 0
        while True:
            lo, n = cursor.claim(3, boundary=self.rel.relseg_size)
            if n == 0:
                break
            r = pg_scan.cpu_scan(self.rel, self.cfg, blocks=(lo, lo + n), **self.pred)
            parts.append(r.items)
            pages += r.pages
        items = np.concatenate(parts) if parts else np.zeros(0, np.uint64)
        return pg_scan.ScanResult(items, pages=pages)

    def close(self):
        pass


def _heap_worker(rank, world, port, path, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        from nvme_strom_amd.models import pg_scan
        import nvme_strom_amd.parallel.scan as PS
        PS.pg_scan.HeapRelationScan = _CpuHeapScan
        dist.init_process_group("gloo")
        rel = pg_scan.Relation(path, relseg_size=8)
        cfg = pg_scan.ScanConfig(chunk_size=4 * 8192, buffer_size=8 * 8192)
        ds = PS.DistributedHeapScan(rel, cfg, torch.device("cpu"), attr_off=0, attr_width=8,
                                    lo=50, hi=1749)
        out = ds.run(1)
        q.put((rank, dict(items=out["items"], counts=out["per_rank_items"],
                          pages=out["totals"]["pages"])))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_distributed_heap_scan_shared_cursor_3_ranks(tmp_path):
    from nvme_strom_amd.models import pg_scan
    from nvme_strom_amd.utils import pgpage
    vals = np.arange(4000, dtype=np.int64)
    data = pgpage.build_table(vals, per_page=100, width=8, invisible_every=10)   # 40 pages
    rel = pg_scan.Relation.write(str(tmp_path / "16390"), data, relseg_size=8)
    cfg = pg_scan.ScanConfig(chunk_size=4 * 8192, buffer_size=8 * 8192)
    full = pg_scan.cpu_scan(rel, cfg, attr_off=0, attr_width=8, lo=50, hi=1749)
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_heap_worker, args=(r, world, port, rel.path, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r], dict), res[r]
        assert np.array_equal(res[r]["items"], full.items), r     # block order, exactly once
        assert sum(res[r]["counts"]) == len(full.items)
        assert res[r]["pages"] == rel.nblocks                    # shared counters: all pages
    assert not any(f.startswith("nvme-strom-scan.dist-") for f in os.listdir("/dev/shm"))
