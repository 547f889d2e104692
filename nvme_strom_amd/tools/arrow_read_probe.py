"""The Arrow scan's reads alone, per read mode, against the storage's own
sequential rate in the same run.

For one column of the config-5 file (tools.arrow_bench.make_file) the scan's
groups are read into their HBM slots — no decode, no filter — as the scan
issues them (a ring of slots, nslots - 1 groups in flight behind the first):

  * ``extents``: MEMCPY_SSD2GPU_EXTENTS of the group's buffers (ArrowScan.EXTENTS)
  * ``chunks``:  MEMCPY_SSD2GPU of the fixed-size chunk ids covering them

``buffer_GBps`` counts the column's buffer bytes (what the scan needs),
``read_GBps`` the bytes the requests read; ``of_storage`` divides the buffer
rate by a host-only io_uring O_DIRECT sequential read of the same file with
the engine's request size, rings and depth, taken before and after;
``of_same_requests`` divides the read rate by the same rings reading exactly
the extents planner's requests (``requests()``, raw_read_list), rep by rep
after the modes — what the storage does with that access pattern.  Rates
are medians over ``--reps`` runs, the file evicted before each.

``python -m nvme_strom_amd.tools.arrow_read_probe --codec zstd --columns val --out p.json``
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


class _Reader:
    """One read mode's prepared groups and slots for a column."""

    def __init__(self, path: str, col: str, mode: str):
        from nvme_strom_amd.models.arrow_scan import ArrowScan
        self.mode = mode
        sc = ArrowScan(path, "cuda")
        sc.EXTENTS = mode == "extents"               # per instance (A/B in one process)
        plan, _, _ = sc._plan([col])
        self.groups = sc._groups(plan)
        sc._ensure_slots(self.groups)
        self.sc = sc
        st = plan.present & (plan.length > 0)
        self.need = int(plan.length[st].sum())
        self.nread = sum(g.read_bytes for g in self.groups)
        self.times, self.submits = [], 0

    def run(self) -> None:
        import nvme_strom_amd as S
        sc = self.sc
        fd = sc.reader.fd
        S.evict_file(fd)
        t0 = time.perf_counter()
        inflight, submits = [], 0
        for k, g in enumerate(self.groups):
            if len(inflight) >= len(sc._slots):
                sc.reader.finish(inflight.pop(0))
            s = sc._slots[k % len(sc._slots)]
            if sc.EXTENTS:
                r = S.memcpy_ssd2gpu_extents(sc._hbm.handle, s.off, fd, g.ext, gap_max=sc.EXTENT_GAP,
                                             sess=sc.reader.sess)
            else:
                r, _ = sc.reader.submit(sc._hbm, s.off, g.ids.astype(np.uint32))
            submits += r.nr_dma_submit
            inflight.append(r)
        for r in inflight:
            sc.reader.finish(r)
        self.times.append(time.perf_counter() - t0)
        self.submits = submits

    def row(self) -> dict:
        med = float(np.median(self.times))
        return dict(mode=self.mode, groups=len(self.groups), buffer_bytes=self.need,
                    bytes_read=self.nread, read_amplification=round(self.nread / max(self.need, 1), 3),
                    requests=self.submits,
                    avg_request_kib=round(self.nread / max(self.submits, 1) / 1024, 1),
                    ms=[round(t * 1e3, 1) for t in self.times],
                    buffer_GBps=round(self.need / med / 1e9, 2),
                    read_GBps=round(self.nread / med / 1e9, 2))


def requests(groups, gap: int, mreq: int, page: int = 4096):
    """(offsets, lengths) of the reads the extents planner issues for the
    groups (tests/test_extents_cpu.py model_layout's runs: page-widened
    extents, holes up to ``gap`` read through), each run cut at
    ``mreq`` — the storage-side comparator's request list."""
    offs, lens = [], []
    for g in groups:
        runs, cur = [], None
        for o, n in zip(g.ext["file_off"].tolist(), g.ext["len"].tolist()):
            if n == 0:
                continue
            a, b = o // page * page, -(-(o + n) // page) * page
            if cur is not None and a <= cur[1] + gap:
                cur[1] = max(cur[1], b)
            else:
                cur = [a, b]
                runs.append(cur)
        for a, b in runs:
            for x in range(a, b, mreq):
                offs.append(x)
                lens.append(min(mreq, b - x))
    return np.array(offs, np.uint64), np.array(lens, np.uint32)


def probe(path: str, col: str, modes, reps: int) -> list:
    """Every mode of ``modes`` on one column, interleaved rep by rep (the
    box's storage rate drifts within a run: a mode's reps in a block would
    take a different storage than the other's)."""
    import nvme_strom_amd as S
    rd = [_Reader(path, col, m) for m in modes]
    # the storage reading the extents planner's own requests, no engine: a
    # column's buffers are 200-500 KiB reads with other columns between them
    # (not the 1 MiB sequential stream storage_seq measures)
    sc = rd[0].sc
    offs, lens = requests(rd[0].groups, sc.EXTENT_GAP, int(S.config_get("max_request")))
    nw, qd = int(S.config_get("workers")), int(S.config_get("queue_depth"))
    same = []
    for _ in range(reps):
        for r in rd:
            r.run()
        S.evict_file(sc.reader.fd)
        same.append(S.raw_read_list(sc.reader.fd, offs, lens, threads=nw, qd=qd, fixed=True)[1]
                    * (1 << 30) / 1e9)
    out = [r.row() for r in rd]
    same_gbps = float(np.median(same))
    for row in out:
        row["same_requests_GBps"] = round(same_gbps, 2)
        row["same_requests"] = len(offs)
        row["of_same_requests"] = round(row["read_GBps"] / same_gbps, 3)
    for r in rd:
        r.sc.close()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="zstd", choices=["lz4", "zstd"])
    ap.add_argument("--columns", default="val")
    ap.add_argument("--rows", type=int, default=1 << 27)
    ap.add_argument("--batch-rows", type=int, default=1 << 16)
    ap.add_argument("--dir", default="/tmp/strom_arrow")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="extents,chunks")
    ap.add_argument("--geometries", default="",
                    help="engine workers x queue depth to sweep, e.g. 4x8,8x16 (default: as configured)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import nvme_strom_amd as S
    from nvme_strom_amd.tools.arrow_bench import make_file
    os.makedirs(a.dir, exist_ok=True)
    tag = "" if a.codec == "lz4" else f"_{a.codec}"
    path = os.path.join(a.dir, f"t_{a.rows}_{a.batch_rows}{tag}.arrow")
    t0 = time.time()
    make_file(path, a.rows, a.batch_rows, codec=a.codec)
    _log(f"file {os.path.getsize(path) >> 20} MiB ready in {time.time() - t0:.1f}s")
    fd = os.open(path, os.O_RDONLY)
    mreq = int(S.config_get("max_request"))
    nw, qd = int(S.config_get("workers")), int(S.config_get("queue_depth"))

    def seq():
        S.evict_file(fd)
        return S.raw_read_rate(fd, mreq, max(64, (2 << 30) // mreq), threads=nw, qd=qd,
                               sequential=True)[1] * (1 << 30) / 1e9
    res = dict(codec=a.codec, rows=a.rows, file_bytes=os.path.getsize(path),
               storage_seq_GBps_before=round(seq(), 2), runs=[])
    geoms = [tuple(int(v) for v in g.split("x")) for g in a.geometries.split(",") if g] or [None]
    for geo in geoms:
        if geo is not None:
            S.configure(workers=geo[0], queue_depth=geo[1])
        for col in a.columns.split(","):
            for row in probe(path, col, a.modes.split(","), a.reps):
                row["column"] = col
                row["workers_qd"] = (f"{S.config_get('workers')}x{S.config_get('queue_depth')}")
                res["runs"].append(row)
                _log(json.dumps(row))
    res["storage_seq_GBps_after"] = round(seq(), 2)
    ceil = max(res["storage_seq_GBps_before"], res["storage_seq_GBps_after"])
    for row in res["runs"]:
        row["of_storage"] = round(row["buffer_GBps"] / ceil, 3)
    os.close(fd)
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
