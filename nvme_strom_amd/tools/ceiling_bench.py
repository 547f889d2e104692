"""Engine ceiling with the storage taken out.

The pool box's storage answers at 22-30 GiB/s, so the headline bench can't
show whether the engine (planner, worker rings, pinned staging, the HBM
ingest grid) would keep up with faster storage — md-raid0 of Gen5 SSDs
(BASELINE config 3) targets a full PCIe Gen5 x16 link.  Here the same
stream (bench shape: 32 MiB segments of 8 KiB chunks, 6 in flight) runs
with ``backend=cache``: every worker read goes through the buffered
descriptor of a file held in the page cache (memory-speed reads), and the
page-cache probe is off so nothing short-cuts the worker + ingest path.
The O_DIRECT run of the same file (page cache evicted) is the storage-bound
reference.  Labelled as an engine ceiling, not a storage number.

``python -m nvme_strom_amd.tools.ceiling_bench --out gpurun_out/ceiling.json``
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-gib", type=float, default=2.0)
    ap.add_argument("--window-mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--workers", default="4,8,16")
    ap.add_argument("--dir", default="/tmp/strom_ceiling")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch

    import nvme_strom_amd as S
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.tensor import HbmBuffer

    os.makedirs(a.dir, exist_ok=True)
    path = os.path.join(a.dir, "ceiling.bin")
    W = a.window_mib << 20
    F = max(W, int(a.file_gib * (1 << 30)) // W * W)
    if not (os.path.exists(path) and os.path.getsize(path) == F):
        rng = np.random.default_rng(5)
        with open(path, "wb") as f:
            for _ in range(F // (64 << 20)):
                f.write(rng.integers(0, 1 << 63, size=(64 << 20) // 8, dtype=np.uint64).tobytes())
            os.fsync(f.fileno())
    with open(path, "rb") as f:
        host_crc = S.crc32c_host(f.read(W))      # window 0, and the page cache warm-up
        while f.read(64 << 20):
            pass
    fd = os.open(path, os.O_RDONLY)
    dev = torch.device("cuda")
    buf = HbmBuffer(W, dev)
    res = dict(file_bytes=F, window_bytes=W, runs={})

    def stream(tag):
        loader = StreamLoader(path, segment_sz=32 << 20, chunk_sz=8192, buf=buf, depth=6)
        ts = []
        for r in range(a.reps + 1):
            if tag == "odirect":
                S.evict_file(fd)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            loader.run((r % (F // W)) * W, W, buf=buf)
            torch.cuda.synchronize()
            if r:
                ts.append(time.perf_counter() - t1)
        loader.run(0, W, buf=buf)
        torch.cuda.synchronize()
        ok = V.crc32c(buf.tensor) == host_crc
        loader.close()
        row = dict(GiBps=round(W / min(ts) / (1 << 30), 2), ms=[round(t * 1e3, 1) for t in ts],
                   verified_crc32c=bool(ok), workers=int(S.config_get("workers")))
        _log(tag, row)
        return row

    try:
        for w in (int(x) for x in a.workers.split(",")):
            S.configure(backend="cache", pgcache_probe=0, workers=w)
            with open(path, "rb") as f:         # re-warm after any eviction
                while f.read(64 << 20):
                    pass
            res["runs"][f"cache_w{w}"] = stream("cache")
        # QD1 4 KiB reads into HBM with the storage taken out: the engine's
        # own latency (lookup, staging, BAR store + flush, completion)
        S.configure(backend="cache", pgcache_probe=0, workers=4)
        offs = np.random.default_rng(1).integers(0, F // 4096, size=1050) * 4096
        lat = S.pread_gpu_latency(buf.handle, 0, fd, offs)[50:] / 1e3
        res["p50_4k_lat_cache_us"] = round(float(np.percentile(lat, 50)), 2)
        res["p99_4k_lat_cache_us"] = round(float(np.percentile(lat, 99)), 2)
        _log("4 KiB QD1 from the page cache: p50 %.2f us" % res["p50_4k_lat_cache_us"])
        S.configure(backend="uring", pgcache_probe=1, workers=4)
        res["runs"]["odirect_w4"] = stream("odirect")
    finally:
        S.configure(backend="uring", pgcache_probe=1, workers=4)
        buf.close()
        os.close(fd)
    res["engine_ceiling_GiBps"] = max(v["GiBps"] for k, v in res["runs"].items()
                                      if k.startswith("cache"))
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
