"""Zstandard decoder (csrc/kernels/zstd.hip) on config-5 streams, next to
the LZ4 decoders on the same columns.

Streams are Arrow IPC buffers exactly as pyarrow writes a 64K-row int64 /
float64 column batch (i64 length + one zstd frame, or one LZ4 frame of
linked 64 KiB blocks for the LZ4 rows): ``val`` (uniform in [0, 1e6) —
arrow_bench's val column), ``ids`` (sorted), ``x`` (uniform float64) and
``text``.  K distinct frames are built on the host; stream i decodes frame
i mod K into its own output.  Every output is verified against the source
bytes on the device.  GB/s = decoded bytes / kernel time (device events),
median of --iters launches.

``python -m nvme_strom_amd.tools.zstd_bench --out gpurun_out/zstd.json``
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def column(kind: str, i: int, rng) -> bytes:
    if kind == "val":
        return rng.integers(0, 1_000_000, 65536, dtype=np.int64).tobytes()
    if kind == "ids":
        return np.arange(i * 65536, (i + 1) * 65536, dtype=np.int64).tobytes()
    if kind == "x":
        return rng.random(65536).tobytes()
    words = [b"select", b"from", b"where", b"gpu", b"hbm", b"nvme", b"strom"]
    return b" ".join(words[j] for j in rng.integers(0, len(words), 110000))[:512 << 10]


def frames(kind: str, k: int, codec: str, level: int, seed: int = 1):
    import pyarrow as pa
    from nvme_strom_amd.ops import decompress as D
    rng = np.random.default_rng(seed)
    raws, bufs = [], []
    for i in range(k):
        d = column(kind, i, rng)
        raws.append(d)
        if codec == "zstd":
            z = pa.Codec("zstd", compression_level=level).compress(d, asbytes=True)
            bufs.append(D.arrow_zstd_buffer(d, z))
        else:
            bufs.append(D.arrow_lz4_buffer(d, pa.compress(d, codec="lz4", asbytes=True)))
    return raws, bufs


PHASES = ("hdr", "copy", "lit_load", "lit_dec", "seq_load", "seq_dec", "fill", "double", "write")
COUNTS = ("chunks", "batches", "double_rounds", "lit_rounds")


def prof(cid, n, src, dst, d_desc, status) -> dict:
    """One launch of the profiled build (libstrom_zstdprof.so): share of
    lane-0 cycles per phase, cycles and events per stream."""
    import ctypes as C
    import os
    from nvme_strom_amd.ops._util import ptr
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(__file__)), "lib",
                              "libstrom_zstdprof.so"))
    out = np.zeros(len(PHASES) + len(COUNTS), dtype=np.uint64)
    lib.strom_zstd_prof(out.ctypes.data_as(C.c_void_p))             # zero
    rc = lib.strom_decompress_zstd(cid, C.c_void_p(ptr(src)), C.c_void_p(ptr(dst)),
                                   C.c_void_p(ptr(d_desc)), C.c_uint32(n),
                                   C.c_void_p(ptr(status)), None, C.c_uint64(0), None)
    assert rc == 0
    lib.strom_zstd_prof(out.ctypes.data_as(C.c_void_p))
    cyc = out[:len(PHASES)].astype(np.float64)
    tot = cyc.sum()
    res = {p: round(float(c / tot), 3) for p, c in zip(PHASES, cyc)}
    res.update({k: round(float(v) / n, 2) for k, v in zip(COUNTS, out[len(PHASES):])})
    res["cycles_per_stream"] = round(float(tot) / n)
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="val,ids,x,text")
    ap.add_argument("--streams", default="256,1024,2048,8192")
    ap.add_argument("--levels", default="1,3")
    ap.add_argument("--distinct", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--no-lz4", dest="lz4", action="store_false",
                    help="skip the LZ4 rows of the same columns")
    ap.add_argument("--prof", action="store_true",
                    help="phase cycle profile of each zstd row (libstrom_zstdprof.so)")
    ap.add_argument("--libs", default="",
                    help="comma list of lib/zv/<name>.so geometry builds (make zv) timed too")
    ap.add_argument("--modes", default="auto,wave,fp",
                    help="zstd decoder choice per row: auto (by stream count), wave (one wave "
                         "per stream), fp (frame-parallel: a frame's blocks on a workgroup's "
                         "waves), lp (lane-parallel: blocks' entropy stages on lanes)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch

    from nvme_strom_amd.ops import decompress as D
    from nvme_strom_amd.ops._util import check, lib, ptr

    dev = torch.device("cuda")
    res = {"lds_bytes_per_stream": int(lib().strom_zstd_lds_bytes()), "rows": []}
    cases = [("zstd", int(l)) for l in a.levels.split(",") if l] + ([("lz4", 0)] if a.lz4 else [])
    import ctypes as C
    import os
    variants = [("lib", None)]
    for v in [x for x in a.libs.split(",") if x]:
        so = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(__file__)), "lib", "zv", v + ".so"))
        so.strom_decompress_zstd.restype = C.c_int
        so.strom_decompress_zstd.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                             C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        so.strom_zstd_lds_bytes.restype = C.c_uint32
        res.setdefault("variant_lds_bytes", {})[v] = int(so.strom_zstd_lds_bytes())
        if hasattr(so, "strom_decompress_zstd_lp"):
            so.strom_decompress_zstd_lp.restype = C.c_int
            so.strom_decompress_zstd_lp.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                                    C.c_uint32, C.c_void_p, C.c_uint64,
                                                    C.c_void_p]
            so.strom_zstd_lp_last.argtypes = [C.c_void_p, C.c_void_p]
        variants.append((v, so))
    for kind in a.kinds.split(","):
        for codec, level in cases:
            raws, bufs = frames(kind, a.distinct, codec, level)
            rawlen = len(raws[0])
            src_off = np.cumsum([0] + [len(b) for b in bufs[:-1]])
            src = torch.from_numpy(np.frombuffer(b"".join(bufs), dtype=np.uint8).copy()).to(dev)
            ref = torch.from_numpy(np.frombuffer(b"".join(raws), dtype=np.uint8).copy()).to(dev)
            ratio = sum(len(b) for b in bufs) / sum(len(r) for r in raws)
            cid = D.ARROW_ZSTD if codec == "zstd" else D.ARROW_LZ4
            for n in [int(x) for x in a.streams.split(",")]:
                idx = np.arange(n) % a.distinct
                cap = (rawlen + 63) // 64 * 64
                descs = D.make_descs_arrays(src_off[idx], np.array([len(bufs[i]) for i in idx]),
                                            np.arange(n) * cap, np.full(n, cap))
                d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
                dst = torch.empty(n * cap, dtype=torch.uint8, device=dev)
                status = torch.empty(n, dtype=torch.int32, device=dev)
                row = dict(kind=kind, codec=codec, level=level if codec == "zstd" else None,
                           streams=n, bytes=n * rawlen, ratio=round(ratio, 3))
                # a variant build runs in lp mode when lp is asked for (its
                # LP geometry is what differs), else in auto
                runs = [(vn, vf, md) for vn, vf in (variants if codec == "zstd" else variants[:1])
                        for md in (a.modes.split(",") if codec == "zstd" and vf is None else
                                   (["lp"] if "lp" in a.modes.split(",") and codec == "zstd"
                                    else ["auto"]))]
                for vname, vfn, mode in runs:
                    lib().strom_zstd_fp_mode({"auto": -1, "wave": 0, "fp": 1, "lp": -1}[mode])
                    times = []
                    ok = True
                    for it in range(a.iters + 1):
                        dst.fill_(0x5a)
                        status.fill_(-99)
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record()
                        if vfn is None and mode == "lp":
                            rc = lib().strom_decompress_zstd_lp(cid, ptr(src), ptr(dst),
                                                                ptr(d_desc), n, ptr(status),
                                                                dst.numel(), None)
                        elif vfn is None:
                            rc = lib().strom_decompress(cid, ptr(src), ptr(dst), ptr(d_desc), n,
                                                        ptr(status), None)
                        elif mode == "lp":
                            rc = vfn.strom_decompress_zstd_lp(cid, ptr(src), ptr(dst), ptr(d_desc),
                                                              n, ptr(status), dst.numel(), None)
                        else:
                            rc = vfn.strom_decompress_zstd(cid, ptr(src), ptr(dst), ptr(d_desc), n,
                                                           ptr(status), None, 0, None)
                        check(rc, codec)
                        e1.record()
                        torch.cuda.synchronize()
                        if it:
                            times.append(e0.elapsed_time(e1) / 1e3)
                        if it == a.iters:                       # verify the last run
                            st = status.cpu().numpy()
                            out = dst.view(n, cap)[:, :rawlen]
                            want = ref.view(a.distinct, rawlen)[torch.from_numpy(idx).to(dev)]
                            ok = bool((st == rawlen).all()) and bool(torch.equal(out, want))
                    lib().strom_zstd_fp_mode(-1)
                    med = float(np.median(times))
                    pre = ("" if mode == "auto" else mode + "_") if vfn is None else vname + "_"
                    row[pre + "GBps"] = round(n * rawlen / med / 1e9, 2)
                    row[pre + "ms"] = round(med * 1e3, 3)
                    row[pre + "verified"] = ok
                    if mode == "lp":
                        # streams the lane-parallel path decoded itself (not the serial fallback)
                        cnt = np.zeros(4, np.uint64)
                        (vfn or lib()).strom_zstd_lp_last(None, cnt.ctypes.data)
                        row[pre + "lp_blocks"], row[pre + "lp_streams"] = int(cnt[0]), int(cnt[1])
                if a.prof and codec == "zstd":
                    row["phases"] = prof(cid, n, src, dst, d_desc, status)
                _log(json.dumps(row))
                res["rows"].append(row)
                del dst
                torch.cuda.empty_cache()
    js = json.dumps(res)
    if a.out:
        with open(a.out, "w") as fo:
            fo.write(js)
    print(js)
    return 0 if all(v for r in res["rows"] for k, v in r.items() if k.endswith("verified")) else 3


if __name__ == "__main__":
    sys.exit(main())
