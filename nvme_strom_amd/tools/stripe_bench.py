"""BASELINE config 3 on a box without md or several SSDs: a native stripe set
(``api.StripeSet``: stripe ``s`` of ``unit`` bytes in member ``s % n``, the
raid0 map of kmod/strom_core.c) streamed into one GPU with the bench shape
(32 MiB segments of 8 KiB chunks, 6 in flight), against one plain file of
the same size on the same storage.  Every member here lives on the box's
one filesystem, so this measures the stripe path's overhead (per-member
request split, concurrent member reads), not SSD aggregation.

``python -m nvme_strom_amd.tools.stripe_bench --out gpurun_out/stripe.json``
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


def _write(path: str, nbytes: int, seed: int) -> None:
    if os.path.exists(path) and os.path.getsize(path) == nbytes:
        return
    rng = np.random.default_rng(seed)
    with open(path, "wb") as f:
        left = nbytes
        while left:
            n = min(64 << 20, left)
            f.write(rng.integers(0, 1 << 63, size=n // 8, dtype=np.uint64).tobytes())
            left -= n
        os.fsync(f.fileno())


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--members", type=int, default=4)
    ap.add_argument("--member-mib", type=int, default=512)
    ap.add_argument("--unit-kib", type=int, default=1024, help="stripe unit")
    ap.add_argument("--window-mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/strom_stripe")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch

    import nvme_strom_amd as S
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.tensor import HbmBuffer

    os.makedirs(a.dir, exist_ok=True)
    unit = a.unit_kib << 10
    msz = (a.member_mib << 20) // unit * unit
    total = msz * a.members
    W = min(a.window_mib << 20, total)
    members = [os.path.join(a.dir, f"m{k}.bin") for k in range(a.members)]
    single = os.path.join(a.dir, "single.bin")
    t0 = time.time()
    for k, p in enumerate(members):
        _write(p, msz, 100 + k)
    _write(single, total, 99)
    _log(f"{a.members} x {msz >> 20} MiB members + {total >> 20} MiB single in {time.time() - t0:.1f}s")
    dev = torch.device("cuda")
    buf = HbmBuffer(W, dev)
    fds = [os.open(p, os.O_RDONLY) for p in members + [single]]

    def evict():
        for fd in fds:
            S.evict_file(fd)

    res = dict(members=a.members, member_bytes=msz, unit=unit, window_bytes=W, runs={})
    ss = S.StripeSet(members, unit)
    try:
        loaders = {name: StreamLoader(src, segment_sz=32 << 20, chunk_sz=8192, buf=buf, depth=6)
                   for name, src in (("single", single), ("stripe", ss))}
        times = {name: [] for name in loaders}
        for r in range(a.reps + 1):          # interleaved; the first round warms up
            for name, loader in loaders.items():
                evict()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                loader.run(0, W, buf=buf)
                torch.cuda.synchronize()
                if r:
                    times[name].append(time.perf_counter() - t1)
        for name, ts in times.items():
            res["runs"][name] = dict(GiBps=round(W / min(ts) / (1 << 30), 2),
                                     ms=[round(t * 1e3, 1) for t in ts])
            _log(name, res["runs"][name])
        # the buffer holds the stripe set's logical bytes [0, W): stripe s
        # comes from member s % n at offset (s // n) * unit
        crc = 0
        for s_ in range(W // unit):
            with open(members[s_ % a.members], "rb") as f:
                f.seek((s_ // a.members) * unit)
                crc = S.crc32c_host(f.read(unit), crc)
        res["stripe_verified_crc32c"] = bool(V.crc32c(buf.tensor) == crc)
        _log("stripe verified", res["stripe_verified_crc32c"])
        for loader in loaders.values():
            loader.close()
    finally:
        ss.close()
        for fd in fds:
            os.close(fd)
        buf.close()
    res["stripe_over_single"] = round(res["runs"]["stripe"]["GiBps"] /
                                      max(res["runs"]["single"]["GiBps"], 1e-9), 3)
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
