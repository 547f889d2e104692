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


def _verify_worker(rank, world, port, path, window, bad_rank, check_every, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        import nvme_strom_amd as S
        from nvme_strom_amd.parallel import ShardedLoader, init_distributed
        S.configure(gpu_emulation=1, workers=2)
        r, w, dev = init_distributed("gloo")

        def corrupt(step, t):
            if r == bad_rank and step == 2:
                t[12345] ^= 0xFF                     # one flipped byte in this rank's slice

        mine = f"{path}.{r}"
        ld = ShardedLoader(mine, window, dev, segment_sz=window // 2, chunk_sz=8192, depth=2,
                           check_every=check_every, on_loaded=corrupt)
        res = {}
        for i in range(3):
            ld.step(i)
        res["ok_last"] = ld.verify(2)               # slice bad_rank corrupted at step 2
        ld.step(3)
        res["ok_clean"] = ld.verify(3)
        rep = ld.report(wall_s=1.0)
        res["report"] = (len(rep["load_GiBps_per_rank"]), len(rep["collective_ms_per_rank"]),
                         rep["steps"])
        ld.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("check_every", [1, 8])
def test_four_rank_allgather_crc_detects_corrupt_slice(tmp_path, check_every):
    """bench.py's integrity branch, 4 gloo ranks: a deliberately corrupted
    slice makes verify() false on EVERY rank; a clean step verifies true."""
    world, window = 4, 128 << 10
    path = str(tmp_path / "shard")
    for r in range(world):
        np.random.default_rng(10 + r).integers(0, 256, 4 * window, dtype=np.uint8).tofile(f"{path}.{r}")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_verify_worker, args=(r, world, port, path, window, 1, check_every, q))
          for r in range(world)]
    [p.start() for p in ps]
    try:
        got = dict(q.get(timeout=180) for _ in ps)
    finally:
        [p.join(timeout=60) for p in ps]
        [p.kill() for p in ps if p.is_alive()]
    for r in range(world):
        assert isinstance(got[r], dict), got[r]
        assert got[r]["ok_last"] is False
        assert got[r]["ok_clean"] is True
        assert got[r]["report"] == (world, world, 4)


def test_fanout_has_no_per_step_host_sync():
    """The per-step path must not read device values back."""
    import inspect
    from nvme_strom_amd.parallel.fanout import ShardedLoader
    for fn in (ShardedLoader.step, ShardedLoader._fan, ShardedLoader._collectives):
        src = inspect.getsource(fn)
        assert ".tolist()" not in src and ".item()" not in src and ".cpu()" not in src.replace(
            "buf.cpu()", ""), fn.__name__
