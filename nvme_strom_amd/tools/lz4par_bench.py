"""Block-parallel LZ4 decoder (csrc/kernels/lz4par.hip) vs the lane-group
decoder (csrc/kernels/decompress.hip) on config-5 streams.

Streams are Arrow IPC LZ4 buffers exactly as pyarrow writes a 64K-row int64
column batch (i64 length + one LZ4 frame of linked 64 KiB blocks): ``val``
(uniform in [0, 1e6) — arrow_bench's val column), ``ids`` (sorted) and
``text``.  K distinct frames are built on the host; stream i decodes frame
i mod K into its own output.  Every output is verified against the source
bytes on the device.  GB/s = decoded bytes / kernel time (device events),
median of --iters launches, both decoders in the same process.

``python -m nvme_strom_amd.tools.lz4par_bench --out gpurun_out/lz4par.json``
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def frames(kind: str, k: int, seed: int = 1, codec: str = "lz4"):
    import pyarrow as pa
    from nvme_strom_amd.ops import decompress as D
    rng = np.random.default_rng(seed)
    raws, bufs = [], []
    words = [b"select", b"from", b"where", b"gpu", b"hbm", b"nvme", b"strom"]
    for i in range(k):
        if kind == "val":
            d = rng.integers(0, 1_000_000, 65536, dtype=np.int64).tobytes()
        elif kind == "ids":
            d = np.arange(i * 65536, (i + 1) * 65536, dtype=np.int64).tobytes()
        elif kind == "chars":
            # a utf8 column's characters: words of 3-24 random letters
            # (arrow_bench's string file) — LZ4 leaves them at ratio ~0.97,
            # one token per ~370 input bytes
            if i == 0 or not hasattr(frames, "_vocab"):
                letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)
                vr = np.random.default_rng(9)
                frames._vocab = [letters[vr.integers(0, 26, int(vr.integers(3, 25)))].tobytes()
                                 for _ in range(20000)]
            d = b"".join(frames._vocab[j] for j in rng.integers(0, 20000, 40000))[:512 << 10]
        else:
            d = b" ".join(words[j] for j in rng.integers(0, len(words), 110000))[:512 << 10]
        raws.append(d)
        if codec == "snappy":       # raw snappy, as Parquet pages carry it
            bufs.append(pa.compress(d, codec="snappy", asbytes=True))
        else:
            bufs.append(D.arrow_lz4_buffer(d, pa.compress(d, codec="lz4", asbytes=True)))
    return raws, bufs


PHASES = ("hdr", "load", "spec", "validate", "count_scan", "fill", "double", "resolve", "write",
          "rawcopy", "expand")
COUNTS = ("windows", "valid_rounds", "batches", "double_rounds")


def prof(n, src, dst, d_desc, status, codec=None) -> dict:
    """One launch of the profiled build: share of thread-0 cycles per phase
    and events per stream."""
    import ctypes as C
    import os
    from nvme_strom_amd.ops import decompress as D
    from nvme_strom_amd.ops._util import ptr
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(__file__)), "lib",
                              "libstrom_decprof.so"))
    out = np.zeros(len(PHASES) + len(COUNTS), dtype=np.uint64)
    lib.strom_lz4par_prof(out.ctypes.data_as(C.c_void_p))           # zero
    rc = lib.strom_decompress_par(codec or D.ARROW_LZ4, C.c_void_p(ptr(src)), C.c_void_p(ptr(dst)),
                                  C.c_void_p(ptr(d_desc)), C.c_uint32(n), C.c_void_p(ptr(status)),
                                  None)
    assert rc == 0
    lib.strom_lz4par_prof(out.ctypes.data_as(C.c_void_p))
    cyc = out[:len(PHASES)].astype(np.float64)
    tot = cyc.sum()
    res = {p: round(float(c / tot), 3) for p, c in zip(PHASES, cyc)}
    res.update({k: round(float(v) / n, 2) for k, v in zip(COUNTS, out[len(PHASES):])})
    res["cycles_per_stream"] = round(float(tot) / n)
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="val,ids,text")
    ap.add_argument("--streams", default="256,1024,2048,8192")
    ap.add_argument("--distinct", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--prof", action="store_true",
                    help="phase cycle profile of the par decoder (libstrom_decprof.so)")
    ap.add_argument("--variants", default="",
                    help="comma list of lib/lz4v/<name>.so geometry builds (make lz4v) to time too")
    ap.add_argument("--no-lanes", dest="lanes", action="store_false")
    ap.add_argument("--codec", default="lz4", choices=("lz4", "snappy"),
                    help="lz4: Arrow IPC LZ4 frames; snappy: raw snappy buffers (pyarrow)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch

    from nvme_strom_amd.ops import decompress as D
    from nvme_strom_amd.ops._util import check, lib, ptr

    dev = torch.device("cuda")
    res = {"rows": []}
    import ctypes as C
    import os
    decoders = ([("lanes", lib().strom_decompress_lanes)] if a.lanes else []) + \
        [("par", lib().strom_decompress_par), ("par512", lib().strom_decompress_par512),
         ("par512b", lib().strom_decompress_par512b),
         ("auto", lib().strom_decompress)]
    for v in [x for x in a.variants.split(",") if x]:
        so = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(__file__)), "lib", "lz4v",
                                 v + ".so"))
        f = so.strom_decompress_par
        f.restype = C.c_int
        f.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                      C.c_void_p]
        decoders.append((v, f))
    for kind in a.kinds.split(","):
        raws, bufs = frames(kind, a.distinct, codec=a.codec)
        cid = D.SNAPPY if a.codec == "snappy" else D.ARROW_LZ4
        rawlen = len(raws[0])
        src_off = np.cumsum([0] + [len(b) for b in bufs[:-1]])
        src = torch.from_numpy(np.frombuffer(b"".join(bufs), dtype=np.uint8).copy()).to(dev)
        ref = torch.from_numpy(np.frombuffer(b"".join(raws), dtype=np.uint8).copy()).to(dev)
        ratio = sum(len(b) for b in bufs) / sum(len(r) for r in raws)
        for n in [int(x) for x in a.streams.split(",")]:
            idx = np.arange(n) % a.distinct
            cap = (rawlen + 63) // 64 * 64
            descs = D.make_descs_arrays(src_off[idx], np.array([len(bufs[i]) for i in idx]),
                                        np.arange(n) * cap, np.full(n, cap))
            d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
            dst = torch.empty(n * cap, dtype=torch.uint8, device=dev)
            status = torch.empty(n, dtype=torch.int32, device=dev)
            row = dict(kind=kind, codec=a.codec, streams=n, bytes=n * rawlen, ratio=round(ratio, 3))
            for name, f in decoders:
                fn = name
                times = []
                ok = True
                for it in range(a.iters + 1):
                    dst.fill_(0x5a)
                    status.fill_(-99)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    check(f(cid, ptr(src), ptr(dst), ptr(d_desc), n, ptr(status), None), fn)
                    e1.record()
                    torch.cuda.synchronize()
                    if it:
                        times.append(e0.elapsed_time(e1) / 1e3)
                    if it == a.iters:                       # verify the last run
                        st = status.cpu().numpy()
                        out = dst.view(n, cap)[:, :rawlen]
                        want = ref.view(a.distinct, rawlen)[torch.from_numpy(idx).to(dev)]
                        ok = bool((st == rawlen).all()) and bool(torch.equal(out, want))
                med = float(np.median(times))
                row[f"{name}_GBps"] = round(n * rawlen / med / 1e9, 2)
                row[f"{name}_ms"] = round(med * 1e3, 3)
                row[f"{name}_verified"] = ok
            if a.lanes:
                row["speedup"] = round(row["par_GBps"] / row["lanes_GBps"], 2)
            if a.prof:
                row["par_phases"] = prof(n, src, dst, d_desc, status, cid)
            _log(json.dumps(row))
            res["rows"].append(row)
            del dst
            torch.cuda.empty_cache()
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as fo:
            fo.write(js)
    print(js)
    ok = all(v for r in res["rows"] for k, v in r.items() if k.endswith("_verified"))
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
