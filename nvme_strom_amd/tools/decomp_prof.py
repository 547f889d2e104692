"""Where the LZ4/snappy decoder's time goes (csrc/kernels/decompress.hip
built with -DSTROM_DECOMP_PROF into lib/libstrom_decprof.so).

Runs the kbench corpora through the profiling build under each geometry
(streams per wave 16 / 4 / 1) and reports, per decoded sequence, the shader
cycles a stream spent in each code path (s_memtime spans summed over
streams) and how often the expensive events happen.

``python -m nvme_strom_amd.tools.decomp_prof --out gpurun_out/decprof.json``
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

NAMES = ["seq", "literal", "match_near", "match_short", "match_far", "refill", "flush", "header",
         "far_fence", "n_seq", "n_far", "n_refill", "n_flush", "n_lit_pass", "n_match_pass",
         "steps", "w_iter", "w_fast", "w_slow", "w_loop", "w_slow_iter"]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=16384)
    ap.add_argument("--out", default="")
    ap.add_argument("--lib", default="", help="a profiling build other than lib/libstrom_decprof.so")
    ap.add_argument("--g", default="", help="comma-separated geometries (default: all)")
    ap.add_argument("--arrow", action="store_true",
                    help="config-5 buffers instead: pyarrow LZ4 frames of 65,536 int64 "
                         "uniform in [0, 1e6) (arrow_bench's val column), --blocks streams")
    ap.add_argument("--distinct", type=int, default=1,
                    help="K different blocks per corpus (stream i decodes block i mod K)")
    a = ap.parse_args(argv)
    from nvme_strom_amd.ops import decompress as D
    lib = C.CDLL(os.path.abspath(a.lib) if a.lib else
                 os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                              "libstrom_decprof.so"))
    lib.strom_decompress.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.c_void_p, C.c_void_p]
    lib.strom_decomp_prof.argtypes = [C.c_void_p]
    def corpora(seed):
        rng = np.random.default_rng(seed)
        words = [b"select", b"from", b"where", b"gpu", b"hbm", b"nvme", b"strom"]
        return {
            "words": b" ".join(words[i] for i in rng.integers(0, len(words), 16000))[:64 << 10],
            "ints": np.cumsum(rng.integers(0, 5, 8192)).astype(np.int64).tobytes(),
            "rand3": np.random.default_rng(seed + 1).integers(0, 1_000_000, 8192)
            .astype(np.int64).tobytes(),
        }
    if a.arrow:
        return arrow_rows(lib, a)
    pools = [corpora(1 + k) for k in range(a.distinct)]
    K = a.distinct
    res = {}
    dev = torch.device("cuda")
    for cname in pools[0]:
        blks = [p[cname] for p in pools]
        blk = blks[0]
        comps = [D.lz4_compress(b) for b in blks]
        offs = np.cumsum([0] + [len(c) for c in comps])
        one = b"".join(comps)
        comp = comps[0]
        for nblk in sorted({a.blocks, 1024}):
            reps = (nblk + K - 1) // K
            src = torch.from_numpy(np.frombuffer(one * reps, dtype=np.uint8).copy()).to(dev)
            dst = torch.empty(nblk * len(blk), dtype=torch.uint8, device=dev)
            descs = D.make_descs([((i // K) * len(one) + int(offs[i % K]), len(comps[i % K]),
                                   i * len(blk), len(blk)) for i in range(nblk)])
            d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
            status = torch.empty(nblk, dtype=torch.int32, device=dev)
            gs = (16, 8, 4, 1) if nblk <= 1024 else (16, 8, 32)
            if a.g:
                gs = tuple(int(x) for x in a.g.split(","))
            for g in gs:
                os.environ["STROM_DECOMP_G"] = str(g)
                out = np.zeros(len(NAMES), dtype=np.uint64)
                lib.strom_decompress(D.LZ4, src.data_ptr(), dst.data_ptr(), d_desc.data_ptr(),
                                     nblk, status.data_ptr(), None)
                torch.cuda.synchronize()
                lib.strom_decomp_prof(out.ctypes.data)       # discard the warm-up
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                lib.strom_decompress(D.LZ4, src.data_ptr(), dst.data_ptr(), d_desc.data_ptr(),
                                     nblk, status.data_ptr(), None)
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e)
                lib.strom_decomp_prof(out.ctypes.data)
                ok = bool((status.cpu().numpy() == len(blk)).all()) and \
                    bytes(dst[:len(blk)].cpu().numpy()) == blk
                nseq = max(int(out[9]), 1)
                row = dict(ms=round(ms, 3), GBps=round(nblk * len(blk) / ms / 1e6, 1), ok=ok,
                           ratio=round(len(blk) / len(comp), 2),
                           seq_per_block=round(nseq / nblk, 1),
                           cycles_per_seq={NAMES[i]: round(int(out[i]) / nseq, 1) for i in range(9)},
                           events_per_seq={NAMES[i]: round(int(out[i]) / nseq, 3)
                                           for i in range(10, 16)})
                it = max(int(out[16]), 1)
                row["wave"] = dict(iters=int(out[16]),
                                   fast_cyc_per_iter=round(int(out[17]) / it, 1),
                                   slow_cyc_per_iter=round(int(out[18]) / it, 1),
                                   loop_cyc_per_iter=round(int(out[19]) / it, 1),
                                   slow_iter_frac=round(int(out[20]) / it, 3))
                key = f"{cname}_{nblk}_g{g}"
                res[key] = row
                print(key, json.dumps(row), file=sys.stderr, flush=True)
            os.environ.pop("STROM_DECOMP_G", None)
            del src, dst
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


def _row(out, ms, nbytes, nstreams, ok):
    nseq = max(int(out[9]), 1)
    row = dict(ms=round(ms, 3), GBps=round(nbytes / ms / 1e6, 1), ok=ok,
               seq_per_stream=round(nseq / nstreams, 1),
               cycles_per_seq={NAMES[i]: round(int(out[i]) / nseq, 1) for i in range(9)},
               events_per_seq={NAMES[i]: round(int(out[i]) / nseq, 3) for i in range(10, 16)})
    it = max(int(out[16]), 1)
    row["wave"] = dict(iters=int(out[16]),
                       fast_cyc_per_iter=round(int(out[17]) / it, 1),
                       slow_cyc_per_iter=round(int(out[18]) / it, 1),
                       loop_cyc_per_iter=round(int(out[19]) / it, 1),
                       slow_iter_frac=round(int(out[20]) / it, 3))
    return row


def arrow_rows(lib, a) -> int:
    """Per-path profile of the config-5 column buffers (pyarrow frames)."""
    import pyarrow as pa
    from nvme_strom_amd.ops import decompress as D
    dev = torch.device("cuda")
    K = max(1, a.distinct)
    rng = np.random.default_rng(7)
    raw = [rng.integers(0, 1_000_000, 65536, dtype=np.int64).tobytes() for _ in range(K)]
    frames = [pa.compress(b, codec="lz4", asbytes=True) for b in raw]
    info = D.parse_lz4_frame_header(frames[0])
    comps = [f[info.data_offset:] for f in frames]
    cid = D.LZ4_FRAME_BCS if info.block_checksum else D.LZ4_FRAME
    offs = np.cumsum([0] + [len(c) for c in comps])
    one = b"".join(comps)
    n = a.blocks
    blk = len(raw[0])
    reps = (n + K - 1) // K
    src = torch.from_numpy(np.frombuffer(one * reps, dtype=np.uint8).copy()).to(dev)
    dst = torch.empty(n * blk, dtype=torch.uint8, device=dev)
    descs = D.make_descs([((i // K) * len(one) + int(offs[i % K]), len(comps[i % K]), i * blk, blk)
                          for i in range(n)])
    d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    res = {"ratio": round(sum(map(len, raw)) / sum(map(len, comps)), 3)}
    for g in (a.g.split(",") if a.g else ("16", "4")):
        os.environ["STROM_DECOMP_G"] = g
        out = np.zeros(len(NAMES), dtype=np.uint64)
        lib.strom_decompress(cid, src.data_ptr(), dst.data_ptr(), d_desc.data_ptr(), n,
                             status.data_ptr(), None)
        torch.cuda.synchronize()
        lib.strom_decomp_prof(out.ctypes.data)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        lib.strom_decompress(cid, src.data_ptr(), dst.data_ptr(), d_desc.data_ptr(), n,
                             status.data_ptr(), None)
        e.record()
        torch.cuda.synchronize()
        lib.strom_decomp_prof(out.ctypes.data)
        ok = bool((status.cpu().numpy() == blk).all()) and bytes(dst[:blk].cpu().numpy()) == raw[0]
        res[f"arrow_val_{n}_g{g}"] = row = _row(out, s.elapsed_time(e), n * blk, n, ok)
        print(f"arrow_val_{n}_g{g}", json.dumps(row), file=sys.stderr, flush=True)
    os.environ.pop("STROM_DECOMP_G", None)
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
