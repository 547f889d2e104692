"""End-to-end PostgreSQL heap scan (the reference's application, pgsql/
nvme_strom.c ExecNVMEStromNext): a synthetic relation on disk (1 GiB
segment files, 8 KiB pages of int8 tuples with hint bits), scanned by
``HeapRelationScan`` — chunks read through the engine into an HBM ring, the
GPU heap-page kernel checks visibility, applies ``lo <= attr <= hi`` and
compacts qualifying item pointers — against the reference-shaped CPU scan
(``cpu_scan``: SSD2RAM-style reads + host tuple walk) of the same file.

The relation repeats one block of distinct pages (checksums off: a page
checksum covers its block number); the GPU result is checked against the
CPU scan of that block, replicated.

Per (chunk size, workers) configuration the first run is the cold scan a
query pays (scan object construction: session, HBM ring, pinned buffers,
then the scan), reported as ``cold_ms``; the ``--reps`` runs after it
(storage evicted before each) are warm and reported by their MEDIAN
(``GBps``), not the best.  ``gpu_best_GBps`` is the configuration with the
best warm median.

``python -m nvme_strom_amd.tools.pg_bench --out gpurun_out/pg.json``
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


def _evict_paths(paths) -> None:
    import nvme_strom_amd as S
    for p in paths:
        fd = os.open(p, os.O_RDONLY)
        S.evict_file(fd)
        os.close(fd)


def snapshot_template(npages: int, per_page: int, nav_frac: float, seed: int = 1,
                      page_xid: bool = False):
    """A bulk-loaded relation's pages as a snapshot sees them: rows without
    hint bits (nobody has read them since the load), inserted by committed,
    aborted and still-running transactions, some deleted by committed or
    running ones.  A fraction ``nav_frac`` of the pages is NOT all-visible
    (the others carry PD_ALL_VISIBLE and their VM bit, rows from old
    committed xids).  ``page_xid``: every not-all-visible page was filled
    by one transaction (a COPY / bulk INSERT: one xmin per page) instead of
    a random inserter per row.  Returns (pages, VM bits, snapshot, clog)."""
    from nvme_strom_amd.utils import pgpage
    from nvme_strom_amd.utils.pgmvcc import (CommitLog, Snapshot, XACT_ABORTED, XACT_COMMITTED,
                                             XACT_IN_PROGRESS)
    rng = np.random.default_rng(seed)
    clog = CommitLog(1 << 16, base=0)
    for x in range(3, 1 << 16):
        clog.set(x, XACT_COMMITTED)
    for x in rng.choice(np.arange(2000, 60000), 3000, replace=False).tolist():
        clog.set(x, XACT_ABORTED)
    running = sorted(rng.choice(np.arange(50000, 60000), 40, replace=False).tolist())
    for x in running:
        clog.set(x, XACT_IN_PROGRESS)
    snap = Snapshot(xmin=50000, xmax=60000, xip=running)
    nav = np.zeros(npages, bool)
    nav[rng.permutation(npages)[:int(round(nav_frac * npages))]] = True
    vals = rng.integers(-5000, 5000, npages * per_page)
    pages = []
    for p in range(npages):
        row = vals[p * per_page:(p + 1) * per_page].tolist()
        if nav[p]:
            xmin = (np.full(per_page, rng.integers(1000, 62000)) if page_xid
                    else rng.integers(1000, 62000, per_page)).tolist()
            dele = rng.random(per_page) < 0.1
            xmax = np.where(dele, rng.integers(1000, 62000, per_page), 0).tolist()
            masks = [0 if d else pgpage.HEAP_XMAX_INVALID for d in dele.tolist()]
            ts = [pgpage.tuple_bytes(np.int64(v).tobytes(), infomask=m, xmin=int(x0), xmax=int(x1))
                  for v, m, x0, x1 in zip(row, masks, xmin, xmax)]
            pages.append(pgpage.build_page(ts, with_checksum=False))
        else:
            ts = [pgpage.tuple_bytes(np.int64(v).tobytes(), infomask=pgpage.HEAP_XMAX_INVALID,
                                     xmin=int(x0)) for v, x0 in zip(row, rng.integers(3, 1000, per_page))]
            pages.append(pgpage.build_page(ts, with_checksum=False, all_visible=True))
    return b"".join(pages), ~nav, snap, clog


def snapshot_rows(a, best, res, evict_paths) -> None:
    """The snapshot rows: one relation per fraction of pages
    that are not all-visible (0 / 25 / 100 %), scanned with a snapshot
    through the device check (default) and through the host leg
    (mvcc_device=False, the reference's split) in the same call, both
    verified against cpu_scan of the template; rates are warm medians, as
    for the plain rows, and ``of_all_visible`` divides by the 0 % row."""
    from nvme_strom_amd.models import pg_scan
    per_page = 150
    tp = min(a.template_pages, 2048)
    pred = dict(attr_off=0, attr_width=8, lo=-100, hi=2500)
    rows = {}
    for frac in (0.0, 0.25, 1.0):
        t0 = time.time()
        tmpl, av, snap, clog = snapshot_template(tp, per_page, frac)
        reps = max(1, int(a.gib * (1 << 30)) // len(tmpl))
        path = os.path.join(a.dir, "16390")
        rel = pg_scan.Relation.write(path, tmpl * reps, all_visible=np.tile(av, reps))
        one = pg_scan.Relation.write(os.path.join(a.dir, "16391"), tmpl, all_visible=av)
        _log(f"snapshot relation nav={frac} {rel.nblocks} blocks in {time.time() - t0:.1f}s")
        nbytes = rel.nblocks * 8192
        base = dict(verify_checksum=False, chunk_size=best["chunk_mib"] << 20,
                    buffer_size=8 * best["chunk_mib"] << 20, snapshot=snap, clog=clog)
        ref = pg_scan.cpu_scan(one, pg_scan.ScanConfig(**base), **pred)
        for mode, dev in (("device", True), ("host", False)):
            if mode == "host" and frac == 0.0:
                continue                  # nothing to check: the same path as the device row
            cfg = pg_scan.ScanConfig(mvcc_device=dev, **base)
            times = []
            with pg_scan.HeapRelationScan(rel, cfg, "cuda", **pred) as g:
                evict_paths(rel.segments)
                out = g.run(best["workers"])            # cold, discarded
                for _ in range(a.reps):
                    evict_paths(rel.segments)
                    t1 = time.perf_counter()
                    out = g.run(best["workers"])
                    times.append(time.perf_counter() - t1)
            blk = (out.items >> np.uint64(16)).astype(np.int64)
            ok = (len(out.items) == len(ref.items) * reps
                  and np.array_equal(out.items[blk < tp], ref.items)
                  and out.removed == ref.removed * reps and out.pages == rel.nblocks)
            med = float(np.median(times))
            row = dict(GBps=round(nbytes / med / 1e9, 2), ms=[round(t * 1e3, 1) for t in times],
                       not_all_visible=frac, nr_checked=int(out.nr_checked),
                       removed=int(out.removed), selected=int(len(out.items)),
                       relation_bytes=nbytes, workers=best["workers"],
                       chunk_mib=best["chunk_mib"], verified=bool(ok))
            rows[f"snap_{mode}_nav{int(frac * 100)}"] = row
            _log("snapshot", mode, frac, row)
        for p in rel.segments + one.segments + [rel.segments[0] + "_vm", one.segments[0] + "_vm"]:
            try:
                os.unlink(p)
            except OSError:
                pass
    allvis = rows["snap_device_nav0"]["GBps"]
    for k, r in rows.items():
        r["of_all_visible"] = round(r["GBps"] / allvis, 3) if allvis else None
    res["runs"].update(rows)
    res["snapshot_nav100_of_all_visible"] = rows["snap_device_nav100"]["of_all_visible"]
    res["snapshot_device_over_host_nav100"] = round(
        rows["snap_device_nav100"]["GBps"] / max(rows["snap_host_nav100"]["GBps"], 1e-9), 2)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0, help="relation size")
    ap.add_argument("--template-pages", type=int, default=4096)
    ap.add_argument("--workers", default="2,4", help="participant threads to try")
    ap.add_argument("--chunk-mib", default="32,128",
                    help="nvme_strom.chunk_size values to try (ring = 8 chunks)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-blocks", type=int, default=16384,
                    help="blocks the CPU baseline scans (a prefix: its tuple walk is slow)")
    ap.add_argument("--dir", default="/tmp/strom_pg")
    ap.add_argument("--no-quals", dest="quals", action="store_false",
                    help="skip the qualifier-list rows (10-column relation)")
    ap.add_argument("--no-snapshot", dest="snapshot", action="store_false",
                    help="skip the snapshot rows (0 / 25 / 100 %% of pages not all-visible)")
    ap.add_argument("--snapshot-only", action="store_true",
                    help="only the snapshot rows (and the plain scan they are compared with)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import nvme_strom_amd as S
    from nvme_strom_amd.models import pg_scan
    from nvme_strom_amd.utils import pgpage

    os.makedirs(a.dir, exist_ok=True)
    per_page = 150
    rng = np.random.default_rng(0)
    vals = rng.integers(-5000, 5000, a.template_pages * per_page).astype(np.int64)
    t0 = time.time()
    tmpl = pgpage.build_table(vals, per_page=per_page, width=8, with_checksum=False,
                              invisible_every=9)
    assert len(tmpl) == a.template_pages * 8192
    reps = max(1, int(a.gib * (1 << 30)) // len(tmpl))
    path = os.path.join(a.dir, "16384")
    small = os.path.join(a.dir, "16385")
    rel = pg_scan.Relation.write(path, tmpl * reps)
    one = pg_scan.Relation.write(small, tmpl)
    _log(f"relation {rel.nblocks} blocks ({reps} x {a.template_pages}) in {time.time() - t0:.1f}s")
    cfg = pg_scan.ScanConfig(verify_checksum=False)
    pred = dict(attr_off=0, attr_width=8, lo=-100, hi=2500)
    nbytes = rel.nblocks * 8192

    def evict():
        for seg in rel.segments:
            fd = os.open(seg, os.O_RDONLY)
            S.evict_file(fd)
            os.close(fd)

    ref = pg_scan.cpu_scan(one, cfg, **pred)
    per_tmpl = len(ref.items)
    res = dict(relation_bytes=nbytes, blocks=rel.nblocks, template_pages=a.template_pages,
               selected_per_template=per_tmpl, runs={})
    best = None
    for cm, w in ((int(c), int(x)) for c in a.chunk_mib.split(",") for x in a.workers.split(",")):
        ccfg = pg_scan.ScanConfig(verify_checksum=False, chunk_size=cm << 20, buffer_size=8 * cm << 20)
        times = []
        evict()
        t1 = time.perf_counter()
        g = pg_scan.HeapRelationScan(rel, ccfg, "cuda", **pred)     # cold: construct + scan
        out = g.run(w)
        cold = time.perf_counter() - t1
        for r in range(a.reps):
            evict()
            t1 = time.perf_counter()
            out = g.run(w)
            times.append(time.perf_counter() - t1)
        g.close()
        items = out.items
        # replica k of the template: block numbers shifted by k * template_pages
        blk = (items >> np.uint64(16)).astype(np.int64)
        first = items[blk < a.template_pages]
        ok = (len(items) == per_tmpl * reps and np.array_equal(first, ref.items)
              and out.pages == rel.nblocks and out.bad_pages == 0)
        med = float(np.median(times))
        row = dict(GBps=round(nbytes / med / 1e9, 2), ms=[round(t * 1e3, 1) for t in times],
                   cold_ms=round(cold * 1e3, 1), GBps_cold=round(nbytes / cold / 1e9, 2),
                   workers=w, chunk_mib=cm, selected=int(len(items)), verified=bool(ok))
        res["runs"][f"gpu_c{cm}_w{w}"] = row
        _log("gpu", row)
        if best is None or row["GBps"] > best["GBps"]:
            best = row
    res["gpu_best_GBps"] = best["GBps"]            # best configuration's warm median
    res["gpu_best_cold_ms"] = best["cold_ms"]
    if a.snapshot:
        snapshot_rows(a, best, res, evict_paths=_evict_paths)
    # qualifier lists over a 10-column relation of the same size (NULLs,
    # short / long / TOASTed text before the predicated columns): every tuple
    # deformed on the GPU (strom_heap_scan2), at the best configuration above
    if a.quals and not a.snapshot_only:
        from nvme_strom_amd.utils import pgtuple as T
        desc, rows = T.synthetic(a.template_pages * 56, seed=4)
        tmpl2 = T.build_pages(rows, desc, with_checksum=False)
        reps2 = max(1, int(a.gib * (1 << 30)) // len(tmpl2))
        rel2 = pg_scan.Relation.write(os.path.join(a.dir, "16386"), tmpl2 * reps2)
        one2 = pg_scan.Relation.write(os.path.join(a.dir, "16387"), tmpl2)
        n2 = rel2.nblocks * 8192
        t_pages = len(tmpl2) // 8192
        qsets = {"quals1": [T.Qual("a", "between", (-200_000, 300_000))],
                 "quals2": [T.Qual("a", "between", (-500_000, 200_000)),
                            T.Qual("b", "between", (0.1, 0.6))],
                 # CNF: three OR-groups over int / IN-list / text-IN (with a
                 # constant past 32 bytes) / float / null tests
                 "cnf3": [T.Or(T.Qual("a", "between", (-500_000, 300_000)),
                               T.Qual("c", "in", (list(range(1, 12)),))),
                          T.Or(T.Qual("name", "text_in", (["k17", "k3", "k42", "x" * 40],)),
                               T.Qual("b", "between", (0.1, 0.9))),
                          T.Or(T.Qual("e", "between", (-1.0, 1.0)), T.Qual("tail", "isnull"))]}
        ccfg = pg_scan.ScanConfig(verify_checksum=False, chunk_size=best["chunk_mib"] << 20,
                                  buffer_size=8 * best["chunk_mib"] << 20)
        for name, qs in qsets.items():
            ref2 = pg_scan.cpu_scan(one2, cfg, desc=desc, quals=qs)
            g = pg_scan.HeapRelationScan(rel2, ccfg, "cuda", desc=desc, quals=qs)
            for seg in rel2.segments:
                fd = os.open(seg, os.O_RDONLY)
                S.evict_file(fd)
                os.close(fd)
            t1 = time.perf_counter()
            out = g.run(best["workers"])
            cold = time.perf_counter() - t1
            times = []
            for r in range(a.reps):
                for seg in rel2.segments:
                    fd = os.open(seg, os.O_RDONLY)
                    S.evict_file(fd)
                    os.close(fd)
                t1 = time.perf_counter()
                out = g.run(best["workers"])
                times.append(time.perf_counter() - t1)
            g.close()
            blk2 = (out.items >> np.uint64(16)).astype(np.int64)
            ok = (len(out.items) == len(ref2.items) * reps2 and
                  np.array_equal(out.items[blk2 < t_pages], ref2.items) and out.pages == rel2.nblocks)
            med = float(np.median(times))
            row = dict(GBps=round(n2 / med / 1e9, 2), ms=[round(t * 1e3, 1) for t in times],
                       cold_ms=round(cold * 1e3, 1), workers=best["workers"],
                       chunk_mib=best["chunk_mib"], quals=sum(len(c) for c in T.clauses(qs)),
                       clauses=len(qs), selected=int(len(out.items)),
                       relation_bytes=n2, verified=bool(ok),
                       of_single_predicate=round(n2 / med / 1e9 / best["GBps"], 3))
            res["runs"][f"gpu_{name}"] = row
            _log("gpu", name, row)
        q1 = res["runs"].get("gpu_quals1")
        if q1 and q1["GBps"]:
            res["runs"]["gpu_cnf3"]["of_quals1"] = round(res["runs"]["gpu_cnf3"]["GBps"] / q1["GBps"], 3)
        for p in rel2.segments + one2.segments:
            try:
                os.unlink(p)
            except OSError:
                pass
    # the same bytes as a plain stream into HBM (bench shape), same storage
    # state: the I/O ceiling the scan runs against
    import torch
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import HbmBuffer
    seg_bytes = os.path.getsize(rel.segments[0])
    hb = HbmBuffer(seg_bytes, "cuda")
    ts = []
    for r in range(3):
        evict()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for sp in rel.segments:
            ld = StreamLoader(sp, segment_sz=32 << 20, chunk_sz=8192, buf=hb, depth=6)
            ld.run(0, os.path.getsize(sp), buf=hb)
            ld.close()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t1)
    hb.close()
    res["stream_same_files_GBps"] = round(nbytes / float(np.median(ts)) / 1e9, 2)
    _log("stream of the same files", res["stream_same_files_GBps"])
    evict()
    nb_cpu = min(rel.nblocks, a.cpu_blocks)
    t1 = time.perf_counter()
    c = pg_scan.cpu_scan(rel, cfg, blocks=(0, nb_cpu), **pred)
    dt = time.perf_counter() - t1
    res["runs"]["cpu"] = dict(GBps=round(nb_cpu * 8192 / dt / 1e9, 3), ms=round(dt * 1e3, 1),
                              blocks=nb_cpu, selected=int(len(c.items)),
                              equal_to_gpu_prefix=bool(np.array_equal(
                                  c.items, items[blk < nb_cpu])))
    _log("cpu", res["runs"]["cpu"])
    res["gpu_over_cpu"] = round(best["GBps"] / max(res["runs"]["cpu"]["GBps"], 1e-9), 2)
    for p in rel.segments + one.segments:
        try:
            os.unlink(p)
        except OSError:
            pass
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
