"""Block-size sweep, 4 KiB - 4 MiB (BASELINE config 2).

For each block size B the engine's request limit is set to B (every storage
read is at most B bytes, the reference's merge cap, kmod/nvme_strom.c:119-125)
and the file is streamed into HBM with the nvme_test shape (32 MiB segments,
6 in flight, chunk = min(B, 8 KiB); utils/nvme_test.c:40-41, 383-498):

  GiBps        whole-window throughput (page cache evicted first)
  iops         completed storage requests per second during that stream
  p50/p99_us   QD1 latency of single B-byte reads into HBM (native loop)
  raw_*        the storage ceiling for B: the same number of io_uring rings,
               as deep, reading B-byte O_DIRECT blocks into host RAM in file
               order (no engine, no HBM) — the engine's target at that size
               (raw_random_GiBps: the same at random aligned offsets)

``--engine-only``: the same sweep with the storage taken out
(``backend=cache``: the workers read a file held in the page cache through
its buffered descriptor, residency probe off so every chunk still takes the
worker + staging + HBM-ingest path).  Each size then has a real engine
ceiling — GiB/s, IOPS and QD1 p50/p99 of the engine alone — and ``raw_*`` is
the same rings reading the cached file into host RAM.

``--ab KEY`` runs every size twice, KEY=0 and KEY=1 interleaved (e.g.
``--ab fixed_bufs``: io_uring registered staging + READ_FIXED vs plain READ);
``--ab KEY=v1,v2,..`` takes those values (e.g. ``--ab workers=4,8,16``).

``python -m nvme_strom_amd.tools.sweep --out gpurun_out/sweep.json``
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def _mk(path: str, nbytes: int) -> None:
    if os.path.exists(path) and os.path.getsize(path) == nbytes:
        return
    rng = np.random.default_rng(11)
    with open(path, "wb") as f:
        left = nbytes
        while left:
            n = min(64 << 20, left)
            f.write(rng.integers(0, 1 << 63, size=n // 8, dtype=np.uint64).tobytes())
            left -= n
        os.fsync(f.fileno())


def _summary(rows, ab):
    """Median GiB/s, IOPS and p50 per (block, arm) over the repetitions."""
    out = {}
    for r in rows:
        out.setdefault((r["block"], r.get(ab) if ab else None), []).append(r)
    res = []
    for (b, v), rs in sorted(out.items(), key=lambda kv: (kv[0][0], kv[0][1] or 0)):
        med = lambda k: float(np.median([x[k] for x in rs]))
        res.append(dict(block=b, arm=v, n=len(rs), GiBps=round(med("GiBps"), 2),
                        iops=round(med("iops")), p50_us=round(med("p50_us"), 2),
                        p99_us=round(med("p99_us"), 2)))
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-gib", type=float, default=2.0)
    ap.add_argument("--dir", default="/tmp/strom_sweep")
    ap.add_argument("--blocks", default="4K,8K,16K,32K,64K,128K,256K,512K,1M,2M,4M")
    ap.add_argument("--max-gib", type=float, default=1.0, help="bytes streamed per block size (cap)")
    ap.add_argument("--lat-samples", type=int, default=300)
    ap.add_argument("--qd", type=int, default=0, help="engine queue depth override (0 = default)")
    ap.add_argument("--device", default="cuda", help="cpu = emulated HBM (tests)")
    ap.add_argument("--no-raw", dest="raw", action="store_false",
                    help="skip the raw io_uring ceiling per block size")
    ap.add_argument("--engine-only", action="store_true",
                    help="backend=cache: page-cache reads through the full engine path")
    ap.add_argument("--ab", default="",
                    help="config key to A/B at every size: KEY (0 vs 1) or KEY=v1,v2,..")
    ap.add_argument("--reps", type=int, default=1, help="repetitions of every (size, arm)")
    ap.add_argument("--prof", action="store_true",
                    help="per-worker phase attribution of every stream (io_prof)")
    ap.add_argument("--no-lat", dest="lat", action="store_false", help="skip the QD1 latency")
    ap.add_argument("--set", default="", help="extra config for every run: k=v,k=v")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    arms = (None,)
    if a.ab:
        key, _, vals = a.ab.partition("=")
        a.ab = key
        arms = tuple(int(v) for v in vals.split(",")) if vals else (0, 1)

    import torch

    import nvme_strom_amd as S

    def sync():
        if a.device != "cpu":
            torch.cuda.synchronize()
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader

    def size(s: str) -> int:
        m = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
        return int(s[:-1]) * m[s[-1]] if s[-1] in m else int(s)

    os.makedirs(a.dir, exist_ok=True)
    path = os.path.join(a.dir, "sweep.bin")
    F = int(a.file_gib * (1 << 30)) // (4 << 20) * (4 << 20)
    _mk(path, F)
    fd = os.open(path, os.O_RDONLY)
    extra = dict(kv.split("=", 1) for kv in a.set.split(",") if kv)
    keys = ["max_request", "queue_depth", "backend", "pgcache_probe", "io_prof"] + \
        ([a.ab] if a.ab else []) + [k for k in extra if k != a.ab]
    defaults = {k: S.config_get(k) for k in keys}
    evict = (lambda f: None) if a.engine_only else S.evict_file
    if extra:
        S.configure(**extra)
    if a.prof:
        S.configure(io_prof=1)
    if a.engine_only:
        S.configure(backend="cache", pgcache_probe=0)
        with open(path, "rb") as f:                 # hold the file in the page cache
            while f.read(64 << 20):
                pass
    rows = []
    sizes = [size(x) for x in a.blocks.split(",")]
    # interleaved arms, --reps times each (the box's storage drifts)
    runs = [(B, v) for B in sizes for _ in range(a.reps) for v in arms]
    try:
        for B, abv in runs:
            kv = {"max_request": B}
            if a.qd:
                kv["queue_depth"] = a.qd
            if a.ab:
                kv[a.ab] = abv
            S.configure(**kv)
            chunk = min(B, 8192)
            nbytes = min(int(a.max_gib * (1 << 30)), B * 65536, F) // (32 << 20) * (32 << 20)
            nbytes = max(nbytes, 32 << 20)
            ld = StreamLoader(path, segment_sz=32 << 20, nr_segments=6, chunk_sz=chunk,
                              device=a.device, depth=6)
            evict(fd)
            ld.run(0, 32 << 20)                      # warm the engine, not the cache
            evict(fd)
            sync()
            if a.prof:
                S.io_prof(reset=True)
            st = ld.run(0, nbytes)
            sync()
            prof = S.io_prof() if a.prof else None
            gibs = nbytes / st.seconds / (1 << 30)
            iops = st.nr_submit / st.seconds
            # QD1 latency of B-byte reads at random aligned offsets
            ns = np.zeros(1)
            if a.lat:
                evict(fd)
                rng = np.random.default_rng(B)
                offs = rng.integers(0, F // B, size=a.lat_samples + 20) * B
                ns = S.pread_gpu_latency(ld.buf.handle, 0, fd, offs, B)[20:] / 1e3
            row = dict(block=B, GiBps=round(gibs, 2), iops=round(iops), bytes=nbytes,
                       **({a.ab: abv} if a.ab else {}),
                       avg_req_kib=round(0.5 * st.nr_blocks / st.nr_submit, 1) if st.nr_submit else 0,
                       ram_chunks=st.nr_ram, p50_us=round(float(np.percentile(ns, 50)), 2),
                       p99_us=round(float(np.percentile(ns, 99)), 2))
            if prof:
                row["prof"] = prof
            if a.raw:
                nraw = max(2000, min(nbytes // B, 200000))
                kw = dict(threads=int(S.config_get("workers")), qd=int(S.config_get("queue_depth")))
                # engine-only: the same rings read the cached file (buffered)
                kw["buffered"] = a.engine_only
                evict(fd)
                riops, rgib = S.raw_read_rate(fd, B, nraw, sequential=True, **kw)
                # registered 2 MiB-page buffers (READ_FIXED, as the engine's
                # pinned staging): the better one is the ceiling
                evict(fd)
                fi, fg = S.raw_read_rate(fd, B, nraw, sequential=True, fixed=True, **kw)
                row.update(raw_plain_GiBps=round(rgib, 2), raw_fixed_GiBps=round(fg, 2))
                if fg > rgib:
                    riops, rgib = fi, fg
                evict(fd)
                _, rgib_rand = S.raw_read_rate(fd, B, nraw, **kw)
                row.update(raw_iops=round(riops), raw_GiBps=round(rgib, 2),
                           raw_random_GiBps=round(rgib_rand, 2),
                           of_raw=round(gibs / rgib, 3) if rgib else None)
            if a.ab:
                row["io"] = S.io_info()
            rows.append(row)
            _log(json.dumps(row))
            ld.close()
    finally:
        S.configure(**defaults)
        os.close(fd)
    out = dict(workers=int(S.config_get("workers")), queue_depth=a.qd or int(defaults["queue_depth"]),
               backend="cache (engine only: storage removed)" if a.engine_only
               else S.config_get("backend"), file_bytes=F, ab=a.ab or None,
               io=S.io_info(), rows=rows, summary=_summary(rows, a.ab))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
