"""HDP flush read-back A/B.

CPU stores through the large BAR land in HBM only after an HDP flush; the
flush register write is posted, and reading it back waits for the flush.
This measures what the read-back costs where it can be paid:

  qd1      p50 / p99 of single 4 KiB pread_gpu into HBM (the synchronous path:
           one BAR write + flush per read) for hdp_sync 0 (posted), 1 (read
           back every write) and 2 (default: posted here, read back per batch)
  batch    4 KiB stream through the workers with the BAR path forced
           (ingest_min=65536), hdp_sync 0 vs 2 (one read-back per batch)

``python -m nvme_strom_amd.tools.hdp_ab --out gpurun_out/hdp.json``
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/strom_hdp")
    ap.add_argument("--samples", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch

    import nvme_strom_amd as S
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import HbmBuffer
    os.makedirs(a.dir, exist_ok=True)
    path = os.path.join(a.dir, "hdp.bin")
    F = 1 << 30
    if not (os.path.exists(path) and os.path.getsize(path) == F):
        rng = np.random.default_rng(9)
        with open(path, "wb") as f:
            for _ in range(F // (64 << 20)):
                f.write(rng.integers(0, 1 << 63, size=(64 << 20) // 8, dtype=np.uint64).tobytes())
    fd = os.open(path, os.O_RDONLY)
    with open(path, "rb") as f:                     # page cache: the engine, not storage
        while f.read(64 << 20):
            pass
    S.configure(backend="cache", pgcache_probe=0)
    res = dict(qd1={}, batch={})
    hb = HbmBuffer(64 << 20, "cuda")
    rng = np.random.default_rng(2)
    for rep in range(a.reps):
        for mode in (0, 1, 2):
            S.configure(hdp_sync=mode)
            offs = rng.integers(0, F // 4096, size=a.samples + 50) * 4096
            ns = S.pread_gpu_latency(hb.handle, 0, fd, offs, 4096)[50:] / 1e3
            res["qd1"].setdefault(str(mode), []).append(
                dict(p50_us=round(float(np.percentile(ns, 50)), 3),
                     p99_us=round(float(np.percentile(ns, 99)), 3)))
        for mode in (0, 2):
            S.configure(hdp_sync=mode, ingest_min=65536, max_request=4096)
            ld = StreamLoader(path, segment_sz=32 << 20, chunk_sz=4096, buf=hb, depth=6)
            ld.run(0, 32 << 20, buf=hb)
            torch.cuda.synchronize()
            st = ld.run(0, 512 << 20, buf=hb)
            torch.cuda.synchronize()
            ld.close()
            res["batch"].setdefault(str(mode), []).append(
                dict(iops=round(st.nr_submit / st.seconds), GiBps=round(st.gib_per_s, 2)))
            S.configure(ingest_min=0, max_request=1 << 20)
        print(json.dumps(res), file=sys.stderr, flush=True)
    hb.close()
    os.close(fd)
    summ = {}
    for k in ("0", "1", "2"):
        summ[f"qd1_p50_us_hdp{k}"] = float(np.median([r["p50_us"] for r in res["qd1"][k]]))
    for k in ("0", "2"):
        summ[f"bar_batch_iops_hdp{k}"] = float(np.median([r["iops"] for r in res["batch"][k]]))
    summ["readback_cost_qd1_us"] = round(summ["qd1_p50_us_hdp1"] - summ["qd1_p50_us_hdp0"], 3)
    res["summary"] = summ
    S.configure(hdp_sync=2, backend="uring", pgcache_probe=1)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
