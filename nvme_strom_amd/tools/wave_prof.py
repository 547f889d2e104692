"""Where the wave-per-stream decoder's time goes (csrc/kernels/
decompress_wave.hip built with -DSTROM_WAVE_PROF into
lib/libstrom_waveprof.so): s_memtime spans per phase and event counts,
summed over waves, reported per decoded unit (LZ4 sequence / snappy
element).

``python -m nvme_strom_amd.tools.wave_prof --out gpurun_out/waveprof.json``
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

NAMES = ["t_parse", "t_lit", "t_par", "t_serial", "t_flush", "t_single", "t_refill", "t_total",
         "n_batch", "n_units", "n_single", "n_serial", "n_par", "n_refill", "n_fence", "n_flush"]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1024,2048")
    ap.add_argument("--distinct", type=int, default=61)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    from nvme_strom_amd.ops import decompress as D
    from nvme_strom_amd.tools.decomp_ab import corpora
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                              "libstrom_waveprof.so"))
    lib.strom_decompress_wave.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                          C.c_void_p, C.c_void_p]
    lib.strom_wave_prof.argtypes = [C.c_void_p]
    dev = torch.device("cuda")
    K = a.distinct
    res = {}
    for codec in ("lz4", "snappy"):
        for cname in ("words", "ints"):
            blks = [corpora(1 + k)[cname] for k in range(K)]
            comps = [D.lz4_compress(b) if codec == "lz4" else D.snappy_compress(b) for b in blks]
            offs = np.cumsum([0] + [len(c) for c in comps])
            one = b"".join(comps)
            blk = len(blks[0])
            for nblk in (int(x) for x in a.streams.split(",")):
                reps = (nblk + K - 1) // K
                src = torch.from_numpy(np.frombuffer(one * reps, dtype=np.uint8).copy()).to(dev)
                dst = torch.empty(nblk * blk, dtype=torch.uint8, device=dev)
                descs = D.make_descs([((i // K) * len(one) + int(offs[i % K]), len(comps[i % K]),
                                       i * blk, blk) for i in range(nblk)])
                d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
                status = torch.empty(nblk, dtype=torch.int32, device=dev)
                cid = D.LZ4 if codec == "lz4" else D.SNAPPY
                out = np.zeros(len(NAMES), dtype=np.uint64)
                for _ in range(2):       # warm-up, then the measured launch
                    lib.strom_wave_prof(out.ctypes.data)
                    lib.strom_decompress_wave(cid, src.data_ptr(), dst.data_ptr(), d_desc.data_ptr(),
                                              nblk, status.data_ptr(), None)
                    torch.cuda.synchronize()
                lib.strom_wave_prof(out.ctypes.data)
                st = status.cpu().numpy()
                assert (st == blk).all(), st[:4]
                r = dict(zip(NAMES, (int(x) for x in out)))
                u = max(1, r["n_units"] + r["n_single"])
                row = {"units": u, "bytes_per_unit": round(nblk * blk / u, 2),
                       "units_per_batch": round(r["n_units"] / max(1, r["n_batch"]), 2),
                       "single_frac": round(r["n_single"] / u, 4),
                       "serial_frac": round(r["n_serial"] / u, 4),
                       "par_frac": round(r["n_par"] / u, 4)}
                for k in NAMES:
                    if k.startswith("t_"):
                        row[k + "_per_unit"] = round(r[k] / u, 1)
                row["refills"] = r["n_refill"]
                row["fences"] = r["n_fence"]
                row["flushes"] = r["n_flush"]
                key = f"{codec}_{cname}_{nblk}"
                res[key] = row
                print(key, row, file=sys.stderr, flush=True)
                del src, dst
    js = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
