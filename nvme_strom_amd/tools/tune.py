"""Engine tuning sweep on the GPU box.

Sections (select with --sections):
  h2d   pinned → HBM copy ceiling, 1 and 4 streams
  ram   storage side only: SSD2RAM into a DMA buffer
  gpu   full SSD→HBM path through StreamLoader over backend/workers/qd/
        request size/staging slots
  lat   4 KiB QD1 latency with the engine's own histogram breakdown
        (io = submit→storage done, copy = storage done→in HBM,
        task = ioctl entry→task done) per backend and worker count

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


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-gib", type=float, default=2.0)
    ap.add_argument("--dir", default="/tmp/strom_tune")
    ap.add_argument("--out", default="")
    ap.add_argument("--sections", default="h2d,ram,gpu,lat")
    ap.add_argument("--workers", default="2,4,8")
    ap.add_argument("--qd", default="4,8")
    ap.add_argument("--req", default="1M,4M")
    ap.add_argument("--slots", default="4,8")
    ap.add_argument("--backends", default="uring,psync")
    a = ap.parse_args(argv)
    secs = set(a.sections.split(","))

    def ints(s):
        out = []
        for x in s.split(","):
            m = 1
            if x.endswith("K"):
                m, x = 1 << 10, x[:-1]
            elif x.endswith("M"):
                m, x = 1 << 20, x[:-1]
            out.append(int(x) * m)
        return out

    import torch
    import nvme_strom_amd as S
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import FileReader, HbmBuffer

    os.makedirs(a.dir, exist_ok=True)
    F = int(a.file_gib * (1 << 30))
    path = os.path.join(a.dir, "tune.bin")
    _mk(path, F)
    fd = os.open(path, os.O_RDONLY)
    res = {}
    W = 1 << 30
    nwin = max(1, F // W)
    backends = a.backends.split(",")
    combos = [c for c in itertools.product(backends, ints(a.workers), ints(a.qd), ints(a.req))
              if not (c[0] == "psync" and c[2] != ints(a.qd)[0])]

    if "h2d" in secs:
        pin = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
        dst = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        res["h2d"] = {}
        for nstreams in (1, 4):
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                per = (1 << 30) // nstreams
                for k, s in enumerate(streams):
                    with torch.cuda.stream(s):
                        dst[k * per:(k + 1) * per].copy_(pin[k * per:(k + 1) * per], non_blocking=True)
                torch.cuda.synchronize()
                res["h2d"][f"streams{nstreams}"] = round(1 / (time.perf_counter() - t0), 2)
        del pin, dst
        _log("h2d", res["h2d"])

    if "ram" in secs:
        res["ram"] = []
        with S.alloc_dma_buffer(W) as db:
            for be, w, qd, mr in combos:
                S.configure(backend=be, workers=w, queue_depth=qd, max_request=mr)
                ch = 8192
                ids = np.arange(0, W // ch, dtype=np.uint32)
                best = 0.0
                for rep in range(2):
                    S.evict_file(fd)
                    t0 = time.perf_counter()
                    tasks = []
                    for c0 in range(0, len(ids), 4096):
                        r = S.memcpy_ssd2ram(db.address + c0 * ch, fd,
                                             ids[c0:c0 + 4096] + (rep % nwin) * (W // ch), ch)
                        tasks.append(r.dma_task_id)
                    for t in tasks:
                        S.memcpy_wait(t)
                    best = max(best, W / (time.perf_counter() - t0) / (1 << 30))
                row = dict(backend=be, workers=w, qd=qd, max_request=mr, GiBps=round(best, 2))
                res["ram"].append(row)
                _log("ram", row)

    if "gpu" in secs:
        res["gpu"] = []
        hb = HbmBuffer(W, "cuda")
        for (be, w, qd, mr), slots in itertools.product(combos, ints(a.slots)):
            S.configure(backend=be, workers=w, queue_depth=qd, max_request=mr, staging_slots=slots)
            ld = StreamLoader(path, segment_sz=32 << 20, chunk_sz=8192, buf=hb, depth=6)
            best = 0.0
            for rep in range(3):
                S.evict_file(fd)
                st = ld.run((rep % nwin) * W, W)
                best = max(best, st.gib_per_s)
            ld.close()
            row = dict(backend=be, workers=w, qd=qd, max_request=mr, slots=slots, GiBps=round(best, 2))
            res["gpu"].append(row)
            _log("gpu", row)
        hb.close()

    if "lat" in secs:
        res["lat"] = []
        hb = HbmBuffer(1 << 20, "cuda")
        for be, w in itertools.product(backends, (1, 4)):
            S.configure(backend=be, workers=w, queue_depth=8, max_request=1 << 20)
            S.evict_file(fd)                    # storage path, not page-cache hits
            rd = FileReader(path, chunk_sz=4096, max_chunks=1)
            rng = np.random.default_rng(0)
            ids = rng.integers(0, F // 4096, 600).astype(np.uint32)
            lat = []
            S.stat_hist(reset=True)
            for j, cid in enumerate(ids):
                t1 = time.perf_counter_ns()
                r, _ = rd.submit(hb, 0, np.array([cid], dtype=np.uint32))
                rd.finish(r)
                if j >= 100:
                    lat.append((time.perf_counter_ns() - t1) / 1e3)
            rd.close()
            h = S.stat_hist()
            row = dict(backend=be, workers=w, p50_us=round(float(np.percentile(lat, 50)), 1),
                       p99_us=round(float(np.percentile(lat, 99)), 1),
                       io_p50_us=round(S.hist_percentile(h["io_ns"], 50) / 1e3, 1),
                       copy_p50_us=round(S.hist_percentile(h["copy_ns"], 50) / 1e3, 1),
                       task_p50_us=round(S.hist_percentile(h["task_ns"], 50) / 1e3, 1))
            res["lat"].append(row)
            _log("lat", row)
        hb.close()
    os.close(fd)
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)


if __name__ == "__main__":
    main()
