"""Engine tuning sweep: separates the storage side (SSD2RAM into a DMA
buffer) from the HBM side (pinned → HBM copies) and sweeps backend, worker
count, queue depth and request size for the full SSD→HBM path.

``python -m nvme_strom_amd.tools.tune --file-gib 2 --out gpurun_out/tune.json``
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time

import numpy as np


def _mk(path, nbytes):
    if os.path.exists(path) and os.path.getsize(path) == nbytes:
        return
    rng = np.random.default_rng(7)
    with open(path, "wb") as f:
        left = nbytes
        while left:
            n = min(64 << 20, left)
            f.write(rng.integers(0, 1 << 63, size=n // 8, dtype=np.uint64).tobytes())
            left -= n
        os.fsync(f.fileno())


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-gib", type=float, default=2.0)
    ap.add_argument("--dir", default="/tmp/strom_tune")
    ap.add_argument("--out", default="")
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args(argv)

    import torch
    import nvme_strom_amd as S
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import HbmBuffer

    os.makedirs(a.dir, exist_ok=True)
    F = int(a.file_gib * (1 << 30))
    path = os.path.join(a.dir, "tune.bin")
    _mk(path, F)
    fd = os.open(path, os.O_RDONLY)
    results = {"h2d": {}, "ram": [], "gpu": []}

    # pinned -> HBM copy ceiling (one and several streams)
    pin = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for nstreams in (1, 4):
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        per = (1 << 30) // nstreams
        for k, s in enumerate(streams):
            with torch.cuda.stream(s):
                dst[k * per:(k + 1) * per].copy_(pin[k * per:(k + 1) * per], non_blocking=True)
        torch.cuda.synchronize()
        results["h2d"][f"streams{nstreams}"] = round(1 / (time.perf_counter() - t0), 2)
    del pin
    print("h2d GiB/s", results["h2d"], file=sys.stderr, flush=True)

    W = 1 << 30
    nwin = max(1, F // W)
    backends = ["uring", "psync"]
    workers = [4, 8, 16] if not a.quick else [8]
    qds = [4, 16] if not a.quick else [16]
    reqs = [256 << 10, 1 << 20, 4 << 20] if not a.quick else [1 << 20]
    # storage side only
    with S.alloc_dma_buffer(W) as db:
        for be, w, qd, mr in itertools.product(backends, workers, qds, reqs):
            if be == "psync" and qd != qds[-1]:
                continue
            S.configure(backend=be, workers=w, queue_depth=qd, max_request=mr)
            ch = 8192
            ids = np.arange(0, W // ch, dtype=np.uint32)
            best = 0.0
            for rep in range(2):
                S.evict_file(fd)
                t0 = time.perf_counter()
                tasks = []
                for c0 in range(0, len(ids), 4096):
                    r = S.memcpy_ssd2ram(db.address + c0 * ch, fd, ids[c0:c0 + 4096] + (rep % nwin) * (W // ch), ch)
                    tasks.append(r.dma_task_id)
                for t in tasks:
                    S.memcpy_wait(t)
                best = max(best, W / (time.perf_counter() - t0) / (1 << 30))
            row = dict(backend=be, workers=w, qd=qd, max_request=mr, GiBps=round(best, 2))
            results["ram"].append(row)
            print("ram", row, file=sys.stderr, flush=True)
    # full SSD -> HBM path
    hb = HbmBuffer(W, "cuda")
    for be, w, qd, mr in itertools.product(backends, workers, qds, reqs):
        if be == "psync" and qd != qds[-1]:
            continue
        for slots in ((4, 8, 16) if not a.quick else (8,)):
            S.configure(backend=be, workers=w, queue_depth=qd, max_request=mr, staging_slots=slots)
            ld = StreamLoader(path, segment_sz=32 << 20, chunk_sz=8192, buf=hb, depth=6)
            best = 0.0
            for rep in range(2):
                S.evict_file(fd)
                st = ld.run((rep % nwin) * W, W)
                best = max(best, st.gib_per_s)
            ld.close()
            row = dict(backend=be, workers=w, qd=qd, max_request=mr, slots=slots, GiBps=round(best, 2))
            results["gpu"].append(row)
            print("gpu", row, file=sys.stderr, flush=True)
    hb.close()
    os.close(fd)
    js = json.dumps(results)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)


if __name__ == "__main__":
    main()
