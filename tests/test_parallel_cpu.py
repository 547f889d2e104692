"""Multi-process fan-out on CPU: 2 ranks over gloo, host-emulated HBM.

Each rank loads its shard windows of a common file through the engine and
all-gathers them (the RCCL path on MI355X uses the same ShardedLoader with
nccl); the gathered bytes must equal the concatenation of every rank's
window.  Also covers broadcast mode and shard_range.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nvme_strom_amd.parallel.fanout import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, window, mode, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        import nvme_strom_amd as S
        from nvme_strom_amd.parallel import ShardedLoader, init_distributed, shard_range
        S.configure(gpu_emulation=1, workers=2)
        r, w, dev = init_distributed("gloo")
        size = os.path.getsize(path)
        lo, ln = shard_range(size, w, r, align=window)
        ld = ShardedLoader(path, window, dev, mode=mode, segment_sz=window // 2, chunk_sz=8192,
                           depth=2, file_offset=lo, file_bytes=ln)
        data = np.fromfile(path, dtype=np.uint8)
        results = []
        for i in range(3):
            ld.step(i)
            ld.flush()
            out = ld.out.numpy().copy()
            if mode == "allgather":
                exp = np.concatenate([data[shard_range(size, w, k, align=window)[0] + (i % (shard_range(size, w, k, align=window)[1] // window)) * window:][:window] for k in range(w)])
            else:
                lo0, ln0 = shard_range(size, w, 0, align=window)
                exp = data[lo0 + (i % (ln0 // window)) * window:][:window]
            results.append(bool(np.array_equal(out, exp)))
        ld.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, results))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("mode", ["allgather", "broadcast"])
def test_sharded_fanout_gloo(tmp_path, mode):
    window = 256 << 10
    path = str(tmp_path / "shards.bin")
    data = np.random.default_rng(0).integers(0, 256, 8 * window, dtype=np.uint8)
    data.tofile(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, path, window, mode, q)) for r in range(2)]
    [p.start() for p in ps]
    got = dict(q.get(timeout=120) for _ in ps)
    [p.join(timeout=60) for p in ps]
    for r in range(2):
        assert got[r] == [True, True, True], got[r]


def test_shard_range():
    total = 10 * (1 << 20) + 5
    ranges = [shard_range(total, 4, r) for r in range(4)]
    assert sum(n for _, n in ranges) == total
    assert all(lo % (1 << 20) == 0 for lo, _ in ranges)
    assert ranges[0][0] == 0 and ranges[-1][0] + ranges[-1][1] == total
