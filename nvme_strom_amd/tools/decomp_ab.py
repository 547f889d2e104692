"""Same-box A/B of LZ4/snappy decoder builds.

Kernel timings move by 10-20% between pool boxes, more than most decoder
changes are worth, so variants are compared inside one process: each
shared library passed on the command line is a standalone build of
csrc/kernels/decompress.hip (``make ab AB=name`` builds the working tree
into lib/ab/name.so); the corpora of kbench run through every library in
alternating order, several rounds, and the median is reported.

``python -m nvme_strom_amd.tools.decomp_ab lib/ab/base.so lib/ab/new.so``
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch


def corpora(seed=1):
    rng = np.random.default_rng(seed)
    words = [b"select", b"from", b"where", b"gpu", b"hbm", b"nvme", b"strom"]
    return {
        "words": b" ".join(words[i] for i in rng.integers(0, len(words), 16000))[:64 << 10],
        "ints": np.cumsum(rng.integers(0, 5, 8192)).astype(np.int64).tobytes(),
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--streams", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--distinct", type=int, default=1,
                    help="K different blocks, stream i decodes block i mod K (kbench: 1, all "
                         "streams identical, so the groups of a wave never diverge)")
    ap.add_argument("--cases", default="", help="e.g. lz4_words,snappy_ints (default: all)")
    ap.add_argument("--arrow", type=int, default=0,
                    help="also N config-5 streams: pyarrow LZ4 frames of 65,536 int64 uniform in "
                         "[0, 1e6) (arrow_bench's val column; 24 %% of matches past 2 KiB)")
    ap.add_argument("--g", default="",
                    help="comma-separated STROM_DECOMP_G values: every build runs under each "
                         "(variants named build@g)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    cases = set(a.cases.split(",")) if a.cases else None
    from nvme_strom_amd.ops import decompress as D
    libs = {}
    for p in a.libs:
        lib = C.CDLL(os.path.abspath(p))
        lib.strom_decompress.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_void_p]
        name = os.path.basename(p).rsplit(".", 1)[0]
        for g in (a.g.split(",") if a.g else [""]):
            libs[f"{name}@{g}" if g else name] = (lib, g)
    dev = torch.device("cuda")
    res = {}
    todo = []
    for codec in ("lz4", "snappy"):
        pools = [corpora(1 + k) for k in range(a.distinct)]
        for dname in pools[0]:
            if cases is not None and f"{codec}_{dname}" not in cases:
                continue
            blks = [p[dname] for p in pools]
            comps = [D.lz4_compress(b) if codec == "lz4" else D.snappy_compress(b) for b in blks]
            todo.append((codec, dname, D.LZ4 if codec == "lz4" else D.SNAPPY, blks, comps, a.streams))
    if a.arrow:
        import pyarrow as pa
        rng = np.random.default_rng(7)
        blks = [rng.integers(0, 1_000_000, 65536, dtype=np.int64).tobytes()
                for _ in range(max(1, a.distinct))]
        frames = [pa.compress(b, codec="lz4", asbytes=True) for b in blks]
        info = D.parse_lz4_frame_header(frames[0])
        comps = [f[info.data_offset:] for f in frames]
        todo.append(("lz4f", "val", D.LZ4_FRAME_BCS if info.block_checksum else D.LZ4_FRAME,
                     blks, comps, a.arrow))
    for codec, dname, cid, blks, comps, n in todo:
            blk = blks[0]
            assert all(len(b) == len(blk) for b in blks)
            K = len(comps)
            offs = np.cumsum([0] + [len(c) for c in comps])
            one = b"".join(comps)
            reps = (n + K - 1) // K
            src = torch.from_numpy(np.frombuffer(one * reps, dtype=np.uint8).copy()).to(dev)
            dst = torch.empty(n * len(blk), dtype=torch.uint8, device=dev)
            descs = D.make_descs([((i // K) * len(one) + int(offs[i % K]), len(comps[i % K]),
                                   i * len(blk), len(blk)) for i in range(n)])
            d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
            status = torch.empty(n, dtype=torch.int32, device=dev)
            times = {k: [] for k in libs}

            def run(lg):
                lib, g = lg
                if g:
                    os.environ["STROM_DECOMP_G"] = g
                else:
                    os.environ.pop("STROM_DECOMP_G", None)
                rc = lib.strom_decompress(cid, src.data_ptr(), dst.data_ptr(), d_desc.data_ptr(),
                                          n, status.data_ptr(), None)
                assert rc == 0, rc

            for name, lib in libs.items():           # warm-up + correctness per build
                dst.zero_()
                run(lib)
                torch.cuda.synchronize()
                ok = bool((status == len(blk)).all().item()) and \
                    bytes(dst[(n - 1) * len(blk):].cpu().numpy()) == blks[(n - 1) % K]
                if not ok:
                    raise SystemExit(f"{name}: wrong output on {codec}/{dname}")
            for r in range(a.rounds):
                order = list(libs.items())
                if r % 2:
                    order.reverse()
                for name, lib in order:
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    run(lib)
                    e.record()
                    torch.cuda.synchronize()
                    times[name].append(s.elapsed_time(e))
            row = {k: round(n * len(blk) / float(np.median(v)) / 1e6, 1) for k, v in times.items()}
            res[f"{codec}_{dname}"] = row
            print(f"{codec}_{dname}", json.dumps(row), file=sys.stderr, flush=True)
            del src, dst
    js = json.dumps({"GBps": res, "streams": a.streams, "rounds": a.rounds, "distinct": a.distinct,
                     "arrow_streams": a.arrow})
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
