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

``--side decode``: the side work is the zstd lane-parallel decoder instead
(37-44 KB of LDS per entropy wave) — whether the ingest grid stays resident
next to an LDS-heavy decode, the case an Arrow ZSTD scan's read / decode
overlap depends on.  ``--calibrate`` sizes the side work to about half a
load on the box at hand.  The load rate is reported per mode: overlap must
not come from slower loads.

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


class Decoder:
    """The LDS-heavy side workload: the lane-parallel zstd decoder
    (csrc/kernels/zstd.hip: its entropy waves take 37-44 KB of LDS each,
    three or four per CU) over ``nstreams`` Arrow-style int64 column frames, ``reps``
    launches per step on the side stream — the co-residency case of an
    Arrow ZSTD scan, whose decode of group i runs while group i+1 loads."""

    def __init__(self, dev, nstreams: int = 512, distinct: int = 16):
        import pyarrow as pa
        from nvme_strom_amd.ops import decompress as D
        self.D = D
        rng = np.random.default_rng(3)
        raws = [rng.integers(0, 1_000_000, 65536, dtype=np.int64).tobytes() for _ in range(distinct)]
        codec = pa.Codec("zstd", compression_level=1)
        bufs = [D.arrow_zstd_buffer(r, codec.compress(r, asbytes=True)) for r in raws]
        self.rawlen = len(raws[0])
        idx = np.arange(nstreams) % distinct
        off = np.cumsum([0] + [len(x) for x in bufs[:-1]])
        cap = (self.rawlen + 63) // 64 * 64
        descs = D.make_descs_arrays(off[idx], np.array([len(bufs[i]) for i in idx]),
                                    np.arange(nstreams) * cap, np.full(nstreams, cap))
        self.src = torch.from_numpy(np.frombuffer(b"".join(bufs), np.uint8).copy()).to(dev)
        self.d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
        self.dst = torch.empty(nstreams * cap, dtype=torch.uint8, device=dev)
        self.status = torch.empty(nstreams, dtype=torch.int32, device=dev)
        self.n = nstreams
        self.ref = torch.from_numpy(np.frombuffer(raws[0], np.uint8).copy()).to(dev)
        self.cap = cap

    def launch(self, stream, reps: int) -> None:
        for _ in range(reps):
            self.D.decompress_async(self.D.ARROW_ZSTD, self.src, self.dst, self.d_desc, self.status,
                                    stream=stream, zstd_mode=self.D.ZSTD_LP)

    def verified(self) -> bool:
        torch.cuda.synchronize()
        return bool((self.status == self.rawlen).all()) and \
            bool(torch.equal(self.dst[:self.rawlen], self.ref))


def run(path: str, window: int, steps: int, n_equiv: int, overlap: bool, gather_reps: int = 1,
        device: str = "cuda", decoder: "Decoder" = None) -> dict:
    """One schedule; returns the report row (times in s).  ``decoder``: the
    side work is ``gather_reps`` zstd decode launches instead of the copy."""
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import HbmBuffer
    dev = torch.device(device)
    bufs = [HbmBuffer(window, dev) for _ in range(2)]
    # the "received" slices of an (N-1)-peer all-gather, as int64 words;
    # gather_reps x as many stand in for a slower fabric.  ONE kernel per
    # step writes them all (a broadcast copy), as one collective call would
    words = window // 8
    rows = 1 if decoder is not None else max(1, n_equiv - 1) * gather_reps
    out = torch.empty((rows, words), dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(device=dev)
    ld = StreamLoader(path, segment_sz=32 << 20, chunk_sz=8192, buf=bufs[0], depth=6)
    nwin = max(1, os.path.getsize(path) // window)
    evs = []
    load_s = 0.0
    pending = None

    def side_work(src):
        if decoder is not None:
            decoder.launch(side, gather_reps)
        else:
            torch.add(src.unsqueeze(0).expand(out.shape), 0, out=out)   # CU copy kernel
    ld.run(0, window, buf=bufs[0])          # warm the engine and the grid
    with torch.cuda.stream(side):           # and load the side kernels' code
        side_work(bufs[0].tensor.view(torch.int64))
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
            side_work(src)
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
    if decoder is not None:
        ok = decoder.verified()
    else:
        ok = bool(torch.equal(out[-1], bufs[(steps - 1) % 2].tensor.view(torch.int64)))
    ld.close()
    for b in bufs:
        b.close()
    ov = min(1.0, max(0.0, (load_s + gather - wall) / gather)) if gather > 0 else None
    return dict(n_equiv=n_equiv, mode="overlap" if overlap else "serial", steps=steps,
                side="decode" if decoder is not None else "copy", reps=gather_reps,
                window=window, load_s=round(load_s, 5), gather_s=round(gather, 5),
                wall_s=round(wall, 5), overlap=round(ov, 3) if ov is not None else None,
                load_GiBps=round(steps * window / load_s / (1 << 30), 2),
                gather_bytes_per_step=out.numel() * 8 if decoder is None else 0, verified=ok)


def calibrate(path: str, window: int, n_equiv: int, decoder: "Decoder" = None,
              target: float = 0.5, device: str = "cuda") -> int:
    """Side-work repetitions that take about ``target`` x one load on THIS
    box: one load timed, one repetition timed, the ratio rounded (>= 1)."""
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import HbmBuffer
    dev = torch.device(device)
    buf = HbmBuffer(window, dev)
    ld = StreamLoader(path, segment_sz=32 << 20, chunk_sz=8192, buf=buf, depth=6)
    ld.run(0, window, buf=buf)
    t = []
    for k in range(2):
        a = time.perf_counter()
        ld.run(k * window % max(window, os.path.getsize(path) // window * window), window, buf=buf)
        t.append(time.perf_counter() - a)
    load = min(t)
    ld.close()
    side = torch.cuda.Stream(device=dev)
    src = buf.tensor.view(torch.int64)
    out = torch.empty((max(1, n_equiv - 1), window // 8), dtype=torch.int64, device=dev)
    g = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            e0.record(side)
            if decoder is not None:
                decoder.launch(side, 1)
            else:
                torch.add(src.unsqueeze(0).expand(out.shape), 0, out=out)
            e1.record(side)
        e1.synchronize()
        g.append(e0.elapsed_time(e1) / 1e3)
    buf.close()
    one = min(g)
    return max(1, int(round(target * load / one))) if one > 0 else 1


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
    ap.add_argument("--side", default="copy", choices=["copy", "decode"],
                    help="side-stream work: a CU copy (all-gather stand-in) or the zstd decoder")
    ap.add_argument("--calibrate", action="store_true",
                    help="repetitions sized to ~0.5 x one load on this box (overrides --gather-reps)")
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
    dec = Decoder(torch.device("cuda")) if a.side == "decode" else None
    for n in (int(x) for x in a.n.split(",")):
        reps = calibrate(path, a.window_mib << 20, n, dec) if a.calibrate else a.gather_reps
        for ov in (m == "overlap" for m in a.modes.split(",")):
            r = run(path, a.window_mib << 20, a.steps, n, ov, reps, decoder=dec)
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
