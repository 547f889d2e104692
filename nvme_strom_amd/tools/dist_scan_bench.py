"""Config 5 over several GPUs: one Arrow IPC file scanned by N ranks (one
process per GPU, parallel/scan.py), every rank ending with the full
selected row ids and projected values.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        -m nvme_strom_amd.tools.dist_scan_bench --out gpurun_out/dist_scan.json

Rank 0 writes the file (arrow_bench's layout) if it is missing; each timed
run starts with the file evicted from the page cache on every rank.  The
combined result is verified against numpy on rank 0.  Reported: the
slowest rank's scan and combine time (median over runs), per-rank bytes
read, and the column GB/s of the whole job.  With one GPU and several
ranks (gloo, collectives staged through host memory) the ranks share the
device: a rehearsal of the multi-rank path, not a scaling number.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 25)
    ap.add_argument("--batch-rows", type=int, default=1 << 16)
    ap.add_argument("--dir", default="/tmp/strom_arrow")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--backend", default="")
    ap.add_argument("--kind", default="arrow", choices=("arrow", "pg"),
                    help="pg: a PostgreSQL relation scanned by DistributedHeapScan (ranks "
                         "share one block cursor)")
    ap.add_argument("--pg-mib", type=int, default=512)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist

    import nvme_strom_amd as S
    from nvme_strom_amd.parallel.scan import DistributedArrowScan
    from nvme_strom_amd.tools.arrow_bench import column_np, make_file

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    backend = a.backend or ("nccl" if ndev >= world else "gloo")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group(backend, device_id=dev)
        else:
            dist.init_process_group(backend)
    os.makedirs(a.dir, exist_ok=True)
    if a.kind == "pg":
        return _pg(a, rank, world, dev, backend)
    path = os.path.join(a.dir, f"t_{a.rows}_{a.batch_rows}.arrow")
    if rank == 0:
        make_file(path, a.rows, a.batch_rows)
    if world > 1:
        dist.barrier()
    quals, proj = [("val", 100_000, 599_999), ("x", 0.25, 0.75)], "id"
    fd = os.open(path, os.O_RDONLY)
    runs = []
    ds = DistributedArrowScan(path, dev)
    try:
        for r in range(a.reps + 1):
            S.evict_file(fd)
            if world > 1:
                dist.barrier()
            out = ds.scan_where(quals, project=proj)
            runs.append((out.seconds["scan_s"], out.seconds["combine_s"], out.seconds["total_s"]))
    finally:
        os.close(fd)
    rows = [np.array(x) for x in zip(*runs[1:])]          # warm runs
    mine = np.array([np.median(rows[0]), np.median(rows[1]), np.median(rows[2]),
                     float(out.bytes_read)])
    if world > 1:
        t = torch.tensor(mine, dtype=torch.float64)
        allr = [torch.zeros_like(t) for _ in range(world)]
        if backend == "nccl":
            t = t.to(dev)
            allr = [x.to(dev) for x in allr]
        dist.all_gather(allr, t)
        allr = np.stack([x.cpu().numpy() for x in allr])
    else:
        allr = mine[None, :]
    ok = None
    if rank == 0:
        m = None
        for name, lo, hi in quals:
            v, valid = column_np(path, name)
            mm = (v >= lo) & (v <= hi)
            if valid is not None:
                mm &= valid
            m = mm if m is None else m & mm
        ref = np.flatnonzero(m)
        ids, _ = column_np(path, proj)
        ok = bool(np.array_equal(out.indices.cpu().numpy(), ref)
                  and np.array_equal(out.values.cpu().numpy(), ids[ref]))
    ds.close()
    if rank == 0:
        total = float(allr[:, 2].max())
        col_bytes = ds.scan.meta.rows.sum() * 8 * 3
        res = dict(world=world, backend=backend if world > 1 else None, devices=ndev,
                   shared_device=world > ndev, rows=int(ds.scan.meta.rows.sum()),
                   selected=out.selected, per_rank_selected=out.per_rank, ranges=out.ranges,
                   scan_ms_per_rank=[round(x * 1e3, 2) for x in allr[:, 0]],
                   combine_ms_per_rank=[round(x * 1e3, 2) for x in allr[:, 1]],
                   bytes_read_per_rank=[int(x) for x in allr[:, 3]],
                   total_ms=round(total * 1e3, 2),
                   column_GBps=round(col_bytes / total / 1e9, 2), verified=ok,
                   first_run_ms=round(runs[0][2] * 1e3, 2))
        js = json.dumps(res)
        if a.out:
            with open(a.out, "w") as f:
                f.write(js)
        print(js, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if (rank != 0 or ok) else 3


def _pg(a, rank: int, world: int, dev, backend: str) -> int:
    """DistributedHeapScan of a synthetic relation; rank 0 verifies."""
    import time

    import torch.distributed as dist

    import nvme_strom_amd as S
    from nvme_strom_amd.models import pg_scan
    from nvme_strom_amd.parallel.scan import DistributedHeapScan
    from nvme_strom_amd.utils import pgpage
    path = os.path.join(a.dir, "16400")
    tmpl_pages = 2048
    reps = max(1, (a.pg_mib << 20) // (tmpl_pages * 8192))
    if rank == 0:
        rng = np.random.default_rng(0)
        vals = rng.integers(-5000, 5000, tmpl_pages * 150).astype(np.int64)
        tmpl = pgpage.build_table(vals, per_page=150, width=8, with_checksum=False,
                                  invisible_every=9)
        pg_scan.Relation.write(path, tmpl * reps)
    if world > 1:
        dist.barrier()
    rel = pg_scan.Relation(path)
    cfg = pg_scan.ScanConfig(verify_checksum=False, chunk_size=32 << 20, buffer_size=256 << 20)
    pred = dict(attr_off=0, attr_width=8, lo=-100, hi=2500)
    ds = DistributedHeapScan(rel, cfg, dev, **pred)
    times = []
    for r in range(a.reps + 1):
        for seg in rel.segments:
            fd = os.open(seg, os.O_RDONLY)
            S.evict_file(fd)
            os.close(fd)
        if world > 1:
            dist.barrier()
        out = ds.run(2)
        times.append(out["seconds"]["total_s"])
    ds.close()
    ok = None
    if rank == 0:
        t0 = time.perf_counter()
        one = pg_scan.Relation.write(os.path.join(a.dir, "16401"), tmpl)
        ref = pg_scan.cpu_scan(one, cfg, **pred).items
        blk = (out["items"] >> np.uint64(16)).astype(np.int64)
        first = out["items"][blk < tmpl_pages]
        ok = bool(len(out["items"]) == len(ref) * reps and np.array_equal(first, ref))
        for sp in one.segments:
            os.unlink(sp)
        res = dict(kind="pg", world=world, backend=backend if world > 1 else None,
                   relation_bytes=rel.nblocks * 8192, items=int(len(out["items"])),
                   per_rank_items=out["per_rank_items"], pages_total=out["totals"]["pages"],
                   warm_median_ms=round(float(np.median(times[1:])) * 1e3, 2),
                   first_run_ms=round(times[0] * 1e3, 2),
                   GBps=round(rel.nblocks * 8192 / float(np.median(times[1:])) / 1e9, 2),
                   verified=ok, verify_s=round(time.perf_counter() - t0, 2))
        js = json.dumps(res)
        if a.out:
            with open(a.out, "w") as f:
                f.write(js)
        print(js, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        for sp in rel.segments:
            os.unlink(sp)
    return 0 if (rank != 0 or ok) else 3


if __name__ == "__main__":
    sys.exit(main())
