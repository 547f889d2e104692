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


if __name__ == "__main__":
    sys.exit(main())
