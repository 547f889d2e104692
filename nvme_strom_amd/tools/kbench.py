"""Throughput of the CDNA4 post-read kernels at production sizes.

``python -m nvme_strom_amd.tools.kbench [--gib 1] [--only crc,scatter,...]``

Each kernel runs on an HBM-resident input (default 1 GiB), timed with HIP
events over several iterations after a warm-up; GB/s counts the bytes the
kernel must read + write.  Run it under ``rocprofv3 --kernel-trace --stats``
for per-kernel device time and under ``--pmc`` for counters.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--only", default="crc,scatter,verify,heap,lz4,snappy,filter",
                    help="also: mvcc (snapshot check), par (LZ4 decoders by stream count)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    only = set(a.only.split(","))
    from nvme_strom_amd.ops import decompress as D
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.ops.colfilter import bitmap_to_indices, column_filter
    from nvme_strom_amd.ops.heapscan import heap_scan
    from nvme_strom_amd.ops.reorder import chunk_scatter
    from nvme_strom_amd.utils import pgpage

    n = int(a.gib * (1 << 30))
    dev = torch.device("cuda")
    res = {}

    def log(k, sec, nbytes):
        res[k] = dict(ms=round(sec * 1e3, 3), GBps=round(nbytes / sec / 1e9, 1))
        print(k, res[k], file=sys.stderr, flush=True)

    buf = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
    if "crc" in only:
        for ch in (8192, 1 << 16, 1 << 20):
            out = torch.empty((n + ch - 1) // ch, dtype=torch.int32, device=dev)
            log(f"crc32c_chunks_{ch}", timed(lambda: V.crc32c_chunks(buf, ch, out=out)), n)
        log("crc32c_full", timed(lambda: V.crc32c(buf)), n)
    if "scatter" in only:
        ch = 8192
        perm = np.random.default_rng(0).permutation(n // ch).astype(np.uint32)
        dst = torch.empty_like(buf)
        pos = torch.from_numpy(perm.view(np.int32)).to(dev)
        log("chunk_scatter_8k", timed(lambda: chunk_scatter(buf, dst, pos, ch)), 2 * n)
        del dst
    if "verify" in only:
        log("verify_pattern", timed(lambda: V.verify_pattern(buf, 0x41424344)), n)
        log("fill_pattern", timed(lambda: V.fill_pattern(buf, 0x41424344)), n)
    if "heap" in only:
        page = pgpage.build_table(np.arange(150 * 64, dtype=np.int64), per_page=150, width=8)
        reps = max(1, n // len(page))
        reps = min(reps, 0xFFFF // 64)          # item ids address <= 65535 pages
        pages = torch.from_numpy(np.frombuffer(page * reps, dtype=np.uint8).copy()).to(dev)
        nb = pages.numel()
        log("heap_scan", timed(lambda: heap_scan(pages, skip_invisible=True)), nb)
        log("heap_scan_checksum_filter",
            timed(lambda: heap_scan(pages, verify_checksum=True, attr_off=0, attr_width=8,
                                    lo=100, hi=5000)), nb)
        del pages
        # tuple descriptor + qualifier lists (strom_heap_scan2): 10 columns
        # with NULLs, short / long / TOASTed text before the predicated ones
        from nvme_strom_amd.ops.heapscan import Program, heap_scan2
        from nvme_strom_amd.utils import pgtuple as T
        desc, rows = T.synthetic(4000, seed=2)
        tmpl = T.build_pages(rows, desc)
        reps = max(1, min(n // len(tmpl), 0xFFFF // (len(tmpl) // 8192)))
        pages = torch.from_numpy(np.frombuffer(tmpl * reps, dtype=np.uint8).copy()).to(dev)
        nb = pages.numel()
        for name, qs in (("heap_scan2_1qual", [T.Qual("a", "between", (-200_000, 300_000))]),
                         ("heap_scan2_2qual", [T.Qual("a", "between", (-500_000, 200_000)),
                                               T.Qual("b", "between", (0.1, 0.6))]),
                         ("heap_scan2_text_eq", [T.Qual("name", "text_eq", ("k17",))]),
                         ("heap_scan2_4qual_last_col", [T.Qual("c", "in", ([1, 2, 3],)),
                                                        T.Qual("d", "notnull"),
                                                        T.Qual("e", "between", (-0.5, 0.5)),
                                                        T.Qual("tail", "between", (0, 50))])):
            # compiled once, as a scan plan is (the program mode uploads it once)
            P = Program(desc, qs)
            log(name, timed(lambda: heap_scan2(pages, desc, P, verify_checksum=True,
                                               skip_invisible=True)), nb)
            # the same list through the program mode (device-memory CNF)
            log(name.replace("heap_scan2_", "heap_scan2_prog_"),
                timed(lambda: heap_scan2(pages, desc, P, verify_checksum=True,
                                         skip_invisible=True, program=True)), nb)
        # a CNF only the program mode takes: (a in range OR c IS NULL) AND b < 0.6
        cnf = [T.Or(T.Qual("a", "between", (-200_000, 300_000)), T.Qual("c", "isnull")),
               T.Qual("b", "lt", (0.6,))]
        P = Program(desc, cnf)
        log("heap_scan2_prog_cnf2", timed(lambda: heap_scan2(pages, desc, P, verify_checksum=True,
                                                             skip_invisible=True)), nb)
        del pages
    if "mvcc" in only:
        _mvcc_rows(n, dev, log)
    rng = np.random.default_rng(1)
    words = [b"select", b"from", b"where", b"gpu", b"hbm", b"nvme", b"strom"]
    datasets = {
        "words": b" ".join(words[i] for i in rng.integers(0, len(words), 16000))[:64 << 10],
        # sorted int64 ids (a typical columnar payload)
        "ints": np.cumsum(rng.integers(0, 5, 8192)).astype(np.int64).tobytes(),
    }
    for codec in ("lz4", "snappy"):
        if codec not in only:
            continue
        for dname, blk in datasets.items():
            comp = D.lz4_compress(blk) if codec == "lz4" else D.snappy_compress(blk)
            nblk = max(1, min(n // len(blk), 16384))
            src = torch.from_numpy(np.frombuffer(comp * nblk, dtype=np.uint8).copy()).to(dev)
            dst = torch.empty(nblk * len(blk), dtype=torch.uint8, device=dev)
            descs = D.make_descs([(i * len(comp), len(comp), i * len(blk), len(blk)) for i in range(nblk)])
            cid = D.LZ4 if codec == "lz4" else D.SNAPPY
            st = D.decompress(cid, src, dst, descs)
            assert (st == len(blk)).all(), st[:4]
            assert bytes(dst[:len(blk)].cpu().numpy()) == blk
            tag = "64k" if dname == "words" else f"{dname}_64k"
            log(f"decompress_{codec}_{tag}_ratio{len(blk) / len(comp):.1f}",
                timed(lambda: D.decompress(cid, src, dst, descs), 3), nblk * len(blk))
            if codec == "lz4" and dname == "words":
                # the same streams under each geometry (streams per wave), and
                # a few-streams launch (an Arrow scan group: ~1k buffers)
                os.environ["STROM_DECOMP_PAR"] = "0"         # lane groups only
                for g in (16, 8, 4, 1):
                    os.environ["STROM_DECOMP_G"] = str(g)
                    log(f"decompress_lz4_64k_g{g}",
                        timed(lambda: D.decompress(cid, src, dst, descs), 3), nblk * len(blk))
                os.environ.pop("STROM_DECOMP_G", None)
                os.environ.pop("STROM_DECOMP_PAR", None)
                few = min(nblk, 1024)
                log(f"decompress_lz4_64k_{few}streams",
                    timed(lambda: D.decompress(cid, src, dst, descs[:few]), 3), few * len(blk))
            del src, dst
            # 61 different blocks (stream i decodes block i mod 61): the groups
            # of a wave diverge as on real data; the rows above decode copies
            # of one block, which keeps a wave's streams in lockstep
            from nvme_strom_amd.tools.decomp_ab import corpora
            blks = [corpora(1 + k)[dname] for k in range(61)]
            comps = [D.lz4_compress(b) if codec == "lz4" else D.snappy_compress(b) for b in blks]
            offs = np.cumsum([0] + [len(c) for c in comps])
            one = b"".join(comps)
            reps = (nblk + 60) // 61
            src = torch.from_numpy(np.frombuffer(one * reps, dtype=np.uint8).copy()).to(dev)
            dst = torch.empty(nblk * len(blk), dtype=torch.uint8, device=dev)
            descs = D.make_descs([((i // 61) * len(one) + int(offs[i % 61]), len(comps[i % 61]),
                                   i * len(blk), len(blk)) for i in range(nblk)])
            st = D.decompress(cid, src, dst, descs)
            assert (st == len(blk)).all(), st[:4]
            assert bytes(dst[len(blk):2 * len(blk)].cpu().numpy()) == blks[1 % 61]
            log(f"decompress_{codec}_{tag}_distinct61",
                timed(lambda: D.decompress(cid, src, dst, descs), 3), nblk * len(blk))
            del src, dst
    if "par" in only:
        _par_rows(D, dev, log)
    if "filter" in only:
        nv = n // 8
        v = torch.randint(-1000, 1000, (nv,), dtype=torch.int64, device=dev)
        log("column_filter_i64", timed(lambda: column_filter(v, -100, 100)), nv * 8)
        bm, cnt = column_filter(v, -100, 100)
        log("bitmap_to_indices", timed(lambda: bitmap_to_indices(bm, nv, cnt)), nv // 8 + cnt * 4)
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)


def _mvcc_rows(n, dev, log):
    """The heap scan's snapshot check (heapscan.hip mvcc_visible) on
    HBM-resident pages of a bulk-loaded relation (no hint bits; committed,
    aborted and running inserters, 10 % deleted: tools.pg_bench
    snapshot_template), every page checked, against the same pages with
    the check off and with the hint-bit rule; and with a qualifier list."""
    from nvme_strom_amd.ops.heapscan import DeviceMvcc, Program, heap_scan, heap_scan2
    from nvme_strom_amd.tools.pg_bench import snapshot_template
    from nvme_strom_amd.utils import pgtuple as T
    tp = 2048
    tmpl, _, snap, clog = snapshot_template(tp, 150, 1.0)
    reps = max(1, min(n // len(tmpl), 0xFFFF // tp))
    pages = torch.from_numpy(np.frombuffer(tmpl * reps, dtype=np.uint8).copy()).to(dev)
    nb = pages.numel()
    dm = DeviceMvcc(snap, clog, device=dev)
    log("heap_scan_all", timed(lambda: heap_scan(pages)), nb)
    log("heap_scan_hints", timed(lambda: heap_scan(pages, skip_invisible=True)), nb)
    log("heap_scan_mvcc", timed(lambda: heap_scan(pages, mvcc=dm)), nb)
    log("heap_scan_mvcc_filter", timed(lambda: heap_scan(pages, mvcc=dm, attr_off=0, attr_width=8,
                                                         lo=-100, hi=2500)), nb)
    desc = T.TupleDesc.of([("v", "int8")])
    P = Program(desc, [T.Qual("v", "between", (-100, 2500))])
    log("heap_scan2_mvcc_1qual", timed(lambda: heap_scan2(pages, desc, P, mvcc=dm)), nb)
    r = heap_scan(pages, mvcc=dm)
    log_counts = dict(selected=r.count, removed=r.removed, recheck=r.recheck)
    print("mvcc counts", log_counts, file=sys.stderr, flush=True)
    del pages
    # a bulk-loaded relation: one inserting transaction per page (its rows'
    # commit-log lookups hit one line), the usual shape after COPY
    tmpl, _, snap, clog = snapshot_template(tp, 150, 1.0, seed=2, page_xid=True)
    pages = torch.from_numpy(np.frombuffer(tmpl * reps, dtype=np.uint8).copy()).to(dev)
    dm = DeviceMvcc(snap, clog, device=dev)
    log("heap_scan_mvcc_page_xid", timed(lambda: heap_scan(pages, mvcc=dm)), nb)
    del pages


def _par_rows(D, dev, log):
    """Lane-group vs block-parallel (lz4par.hip) LZ4 decoder by stream
    count: 61 distinct 64 KiB blocks per corpus, and config-5-shaped streams
    (pyarrow LZ4 frames of 512 KiB, eight linked 64 KiB blocks each)."""
    from nvme_strom_amd.tools.decomp_ab import corpora

    def run(tag, cid, comps, sizes, counts):
        offs = np.cumsum([0] + [len(c) for c in comps])
        one = b"".join(comps)
        osz = np.cumsum([0] + list(sizes))
        k = len(comps)
        for cnt in counts:
            reps = (cnt + k - 1) // k
            src = torch.from_numpy(np.frombuffer(one * reps, dtype=np.uint8).copy()).to(dev)
            dst = torch.empty(int(osz[-1]) * reps, dtype=torch.uint8, device=dev)
            descs = D.make_descs([((i // k) * len(one) + int(offs[i % k]), len(comps[i % k]),
                                   (i // k) * int(osz[-1]) + int(osz[i % k]), sizes[i % k])
                                  for i in range(cnt)])
            total = sum(sizes[i % k] for i in range(cnt))
            for g in ("lanes", "par"):
                os.environ["STROM_DECOMP_PAR"] = "1" if g == "par" else "0"
                st = D.decompress(cid, src, dst, descs)
                assert (st == np.array([sizes[i % k] for i in range(cnt)])).all(), (g, st[:4])
                j = cnt - 1
                lo = (j // k) * int(osz[-1]) + int(osz[j % k])
                assert bytes(dst[lo:lo + 4096].cpu().numpy()) == corpus_out[j % k][:4096]
                log(f"{g}_{tag}_{cnt}streams",
                    timed(lambda: D.decompress(cid, src, dst, descs), 3), total)
            os.environ.pop("STROM_DECOMP_PAR", None)
            del src, dst

    for codec in ("lz4",):
        for dname in ("words", "ints"):
            corpus_out = [corpora(1 + k)[dname] for k in range(61)]
            comps = [D.lz4_compress(b) if codec == "lz4" else D.snappy_compress(b) for b in corpus_out]
            run(f"{codec}_{dname}", D.LZ4 if codec == "lz4" else D.SNAPPY, comps,
                [len(b) for b in corpus_out], (1024, 2048, 4096, 16384))
    try:
        import pyarrow as pa
    except Exception:
        return
    rng = np.random.default_rng(3)
    corpus_out = [np.cumsum(rng.integers(0, 1 << 12, 65536)).astype(np.int64).tobytes()
                  for _ in range(8)]
    frames = [pa.compress(b, codec="lz4", asbytes=True) for b in corpus_out]
    info = D.parse_lz4_frame_header(frames[0])
    comps = [f[info.data_offset:] for f in frames]
    cid = D.LZ4_FRAME_BCS if info.block_checksum else D.LZ4_FRAME
    run("frame512k_ints", cid, comps, [len(b) for b in corpus_out], (512, 2048))


if __name__ == "__main__":
    main()
