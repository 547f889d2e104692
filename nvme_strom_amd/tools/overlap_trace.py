"""Concurrency of the ingest grid and side-stream kernels in a rocprofv3 trace.

``python -m nvme_strom_amd.tools.overlap_trace kernel_trace.csv [--side add] [--md out.md]``

From a ``--kernel-trace`` CSV of ``tools/overlap_bench.py``: the intervals
the persistent ingest grid was resident (one dispatch per launch), the
side-stream kernels (name substring ``--side``, default the elementwise
copy ``add``), how much side-kernel time fell inside a grid interval, and
the queues each ran on.  Side kernels that ran only while no grid was
resident would mean they waited behind it (a shared hardware queue).
"""
from __future__ import annotations

import argparse
import csv
import json
import sys


def merge(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inside(a, b, merged) -> int:
    t = 0
    for x, y in merged:
        lo, hi = max(a, x), min(b, y)
        if hi > lo:
            t += hi - lo
    return t


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--grid", default="ingest_kernel")
    ap.add_argument("--side", default="add")
    ap.add_argument("--md", default="")
    a = ap.parse_args(argv)
    grid, side = [], []
    gq, sq = set(), set()
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            q = r.get("Queue_Id") or r.get("Stream_Id") or ""
            if a.grid in name:
                grid.append((s, e))
                gq.add(q)
            elif a.side in name:
                side.append((s, e))
                sq.add(q)
    mg = merge(grid)
    side_ns = sum(e - s for s, e in side)
    side_in = sum(inside(s, e, mg) for s, e in side)
    starts_in = sum(1 for s, e in side if inside(s, s + 1, mg))
    res = dict(grid_dispatches=len(grid), grid_resident_ms=round(sum(b - a for a, b in mg) / 1e6, 3),
               side_kernels=len(side), side_ms=round(side_ns / 1e6, 3),
               side_ms_while_grid_resident=round(side_in / 1e6, 3),
               side_fraction_concurrent=round(side_in / side_ns, 3) if side_ns else None,
               side_kernels_started_while_grid_resident=starts_in,
               grid_queues=sorted(gq), side_queues=sorted(sq))
    text = json.dumps(res, indent=1)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write("```\n" + text + "\n```\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
