"""nvme_stat in Python (reference utils/nvme_stat.c): engine counters from the
kernel provider (STAT_INFO) or from userspace engines' shared-memory exports
(/dev/shm/nvme-strom.<pid>, written by libstrom).

``python -m nvme_strom_amd.utils.stat [interval] [--pid PID]``
"""
from __future__ import annotations

import argparse
import glob
import os
import sys
import time
from typing import Dict, Optional

import numpy as np

MAGIC = 0x53544F524D535431
HDR = 64
SCALARS = ["nr_ssd2gpu", "clk_ssd2gpu", "nr_setup_prps", "clk_setup_prps", "nr_submit_dma",
           "clk_submit_dma", "nr_wait_dtask", "clk_wait_dtask", "nr_wrong_wakeup",
           "cur_dma_count", "max_dma_count"]
BUCKETS = 48
WORDS = len(SCALARS) + 8 + 3 * BUCKETS


def read_exports(pid: Optional[int] = None) -> Dict[int, dict]:
    """{pid: counters} for every live engine export."""
    out = {}
    for path in glob.glob("/dev/shm/nvme-strom.*"):
        try:
            p = int(path.rsplit(".", 1)[1])
        except ValueError:
            continue
        if pid is not None and p != pid:
            continue
        try:
            os.kill(p, 0)
        except OSError:
            continue
        try:
            raw = np.fromfile(path, dtype=np.uint64, count=HDR // 8 + WORDS)
        except OSError:
            continue
        if len(raw) < HDR // 8 + WORDS or int(raw[0]) != MAGIC:
            continue
        w = raw[HDR // 8:]
        d = {k: int(w[i]) for i, k in enumerate(SCALARS)}
        base = len(SCALARS)
        for i in range(4):
            d[f"nr_debug{i + 1}"] = int(w[base + i])
            d[f"clk_debug{i + 1}"] = int(w[base + 4 + i])
        h = base + 8
        d["io_ns"] = w[h:h + BUCKETS].copy()
        d["copy_ns"] = w[h + BUCKETS:h + 2 * BUCKETS].copy()
        d["task_ns"] = w[h + 2 * BUCKETS:h + 3 * BUCKETS].copy()
        out[p] = d
    return out


def aggregate(exports: Dict[int, dict]) -> dict:
    tot: dict = {}
    for d in exports.values():
        for k, v in d.items():
            tot[k] = tot[k] + v if k in tot else (v.copy() if isinstance(v, np.ndarray) else v)
    return tot


def tsc_hz(sample_s: float = 0.05) -> float:
    import ctypes
    from .. import _native as N
    lib = N.lib()
    from ..api import stat_info
    a = stat_info()["tsc"]
    t0 = time.perf_counter()
    time.sleep(sample_s)
    b = stat_info()["tsc"]
    return (b - a) / (time.perf_counter() - t0)


def main(argv=None) -> int:
    from ..api import hist_percentile
    ap = argparse.ArgumentParser()
    ap.add_argument("interval", nargs="?", type=float, default=0)
    ap.add_argument("--pid", type=int)
    a = ap.parse_args(argv)
    hz = tsc_hz()
    prev = aggregate(read_exports(a.pid))
    if not prev:
        print("no nvme-strom engine found", file=sys.stderr)
        return 1
    if a.interval <= 0:
        for k in SCALARS:
            print(f"{k:16s} {prev[k]}")
        for name in ("io_ns", "copy_ns", "task_ns"):
            h = prev[name]
            print(f"{name:16s} p50={hist_percentile(h, 50) / 1e3:.1f}us p99={hist_percentile(h, 99) / 1e3:.1f}us")
        return 0
    line = 0
    while True:
        time.sleep(a.interval)
        cur = aggregate(read_exports(a.pid))
        if not cur:
            return 0
        if line % 25 == 0:
            print(f"{'req/s':>10} {'avg-dma':>9} {'avg-prps':>9} {'avg-sub':>9} {'avg-wait':>9} {'dma-cur':>8}")
        def mean(i):
            dn = cur[SCALARS[2 * i]] - prev[SCALARS[2 * i]]
            dc = cur[SCALARS[2 * i + 1]] - prev[SCALARS[2 * i + 1]]
            return dc / hz * 1e6 / dn if dn else 0.0
        dreq = cur["nr_ssd2gpu"] - prev["nr_ssd2gpu"]
        print(f"{dreq / a.interval:10.0f} {mean(0):8.1f}u {mean(1):8.1f}u {mean(2):8.1f}u "
              f"{mean(3):8.1f}u {cur['cur_dma_count']:8d}", flush=True)
        prev = cur
        line += 1


if __name__ == "__main__":
    sys.exit(main())
