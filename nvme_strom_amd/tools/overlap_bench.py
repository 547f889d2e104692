"""Load <-> collective overlap on ONE GPU.

``parallel/fanout.py`` overlaps the all-gather of step i (on a side stream)
with the load of step i+1, whose bytes reach HBM through the engine's
persistent ingest grid (csrc/kernels/ingest.hip) on its own stream.  With
the box's 4 hardware queues, a side-stream kernel that landed on the grid's
queue would wait behind the grid until the load ends: the fan-out would
silently serialize.  This tool runs the ShardedLoader step schedule on one
GPU with the collective replaced by device copy kernels on the side stream,
sized like an N-rank all-gather's receive traffic ((N-1) x window through
CUs, as RCCL's copy kernels do), and reports ``fanout.report()``'s overlap
formula: (load + gather - wall) / gather.

  serial   the gather runs on the side stream but is waited for before the
           next load (the formula's zero point)
  overlap  ShardedLoader's schedule: gather i runs while load i+1 does

``python -m nvme_strom_amd.tools.overlap_bench --out gpurun_out/overlap.json``
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def _mk(path: str, nbytes: int) -> None:
    """A random-byte file, written back and dropped from the page cache (so
    loads take the storage path, not the page-cache write-back path)."""
    if not (os.path.exists(path) and os.path.getsize(path) == nbytes):
        rng = np.random.default_rng(5)
        with open(path, "wb") as f:
            left = nbytes
            while left:
                n = min(64 << 20, left)
                f.write(rng.integers(0, 1 << 63, size=n // 8, dtype=np.uint64).tobytes())
                left -= n
            f.flush()
            os.fsync(f.fileno())
    import nvme_strom_amd as S
    fd = os.open(path, os.O_RDONLY)
    S.evict_file(fd)
    os.close(fd)


def run(path: str, window: int, steps: int, n_equiv: int, overlap: bool, gather_reps: int = 1,
        device: str = "cuda") -> dict:
    """One schedule; returns the report row (times in s)."""
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import HbmBuffer
    dev = torch.device(device)
    bufs = [HbmBuffer(window, dev) for _ in range(2)]
    # the "received" slices of an (N-1)-peer all-gather, as int64 words;
    # gather_reps x as many stand in for a slower fabric.  ONE kernel per
    # step writes them all (a broadcast copy), as one collective call would
    words = window // 8
    out = torch.empty((max(1, n_equiv - 1) * gather_reps, words), dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(device=dev)
    ld = StreamLoader(path, segment_sz=32 << 20, chunk_sz=8192, buf=bufs[0], depth=6)
    nwin = max(1, os.path.getsize(path) // window)
    evs = []
    load_s = 0.0
    pending = None
    ld.run(0, window, buf=bufs[0])          # warm the engine and the grid
    with torch.cuda.stream(side):           # and load the copy kernel's code
        torch.add(bufs[0].tensor.view(torch.int64).unsqueeze(0).expand(out.shape), 0, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        buf = bufs[i % 2]
        a = time.perf_counter()
        ld.run((i % nwin) * window, window, buf=buf)
        load_s += time.perf_counter() - a
        src = buf.tensor.view(torch.int64)
        ev = torch.cuda.Event()
        ev.record()
        start = torch.cuda.Event(enable_timing=True)
        done = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            side.wait_event(ev)
            start.record(side)
            torch.add(src.unsqueeze(0).expand(out.shape), 0, out=out)   # CU copy kernel
            done.record(side)
        evs.append((start, done))
        if not overlap:
            done.synchronize()
        if pending is not None:
            pending.synchronize()
        pending = done
    pending.synchronize()
    torch.cuda.current_stream().synchronize()
    wall = time.perf_counter() - t0
    gather = sum(s.elapsed_time(e) for s, e in evs) / 1e3
    ok = bool(torch.equal(out[-1], bufs[(steps - 1) % 2].tensor.view(torch.int64)))
    ld.close()
    for b in bufs:
        b.close()
    ov = min(1.0, max(0.0, (load_s + gather - wall) / gather)) if gather > 0 else None
    return dict(n_equiv=n_equiv, mode="overlap" if overlap else "serial", steps=steps,
                window=window, load_s=round(load_s, 5), gather_s=round(gather, 5),
                wall_s=round(wall, 5), overlap=round(ov, 3) if ov is not None else None,
                load_GiBps=round(steps * window / load_s / (1 << 30), 2),
                gather_bytes_per_step=out.numel() * 8, verified=ok)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/strom_overlap")
    ap.add_argument("--file-gib", type=float, default=2.0)
    ap.add_argument("--window-mib", type=int, default=256)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--n", default="2,8", help="N-equivalents (gather = (N-1) x window)")
    ap.add_argument("--gather-reps", type=int, default=1,
                    help="x as many bytes copied per step (a slower fabric: more gather time)")
    ap.add_argument("--cache", action="store_true",
                    help="backend=cache (page-cache reads: a faster load)")
    ap.add_argument("--modes", default="serial,overlap")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import nvme_strom_amd as S
    os.makedirs(a.dir, exist_ok=True)
    path = os.path.join(a.dir, "overlap.bin")
    F = int(a.file_gib * (1 << 30)) // (4 << 20) * (4 << 20)
    _mk(path, F)
    if a.cache:
        S.configure(backend="cache", pgcache_probe=0)
        with open(path, "rb") as f:
            while f.read(64 << 20):
                pass
    rows = []
    for n in (int(x) for x in a.n.split(",")):
        for ov in (m == "overlap" for m in a.modes.split(",")):
            r = run(path, a.window_mib << 20, a.steps, n, ov, a.gather_reps)
            r["ingest"] = S.ingest_info(0)
            _log(json.dumps(r))
            rows.append(r)
    res = dict(backend=S.config_get("backend"), hw_queues=os.environ.get("GPU_MAX_HW_QUEUES"),
               ingest_prio=S.config_get("ingest_prio"), rows=rows)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
