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
    for fn in (ShardedLoader.step, ShardedLoader._fan, ShardedLoader._collectives,
               ShardedLoader._retire, ShardedLoader._src_crc):
        src = inspect.getsource(fn)
        assert ".tolist()" not in src and ".item()" not in src and ".cpu()" not in src.replace(
            "buf.cpu()", ""), fn.__name__


def _deliver_worker(rank, world, port, path, window, q):
    """4 gloo ranks: (a) a consumer thread pulls every step's gathered output
    (gathered / release) while the loader thread loads and gathers the next
    step; (b) on_gathered delivers every step exactly once; (c) verify_each
    catches a slice corrupted at step 2 — ShardCorruptError on every rank,
    naming step 2 and the corrupting rank."""
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import threading
        import time
        import torch.distributed as dist
        import nvme_strom_amd as S
        from nvme_strom_amd.parallel import ShardedLoader, init_distributed
        from nvme_strom_amd.parallel.fanout import ShardCorruptError
        S.configure(gpu_emulation=1, workers=2)
        r, w, dev = init_distributed("gloo")
        wins = [np.fromfile(f"{path}.{k}", dtype=np.uint8) for k in range(w)]
        nwin = len(wins[0]) // window

        def expect(i):
            j = i % nwin
            return np.concatenate([x[j * window:(j + 1) * window] for x in wins])

        res = {}
        steps = 6
        # (a) pull consumer in a thread
        ld = ShardedLoader(f"{path}.{r}", window, dev, segment_sz=window // 2, chunk_sz=8192,
                           depth=2, out_ring=2, verify_each=True)
        log, ok = [], []

        def consumer():
            for i in range(steps):
                g = ld.gathered(i, timeout=60)
                log.append(("held", i, time.perf_counter()))
                ok.append(bool(np.array_equal(g.tensor.numpy(), expect(i))))
                time.sleep(0.15)                   # hold it while the next step runs
                log.append(("released", i, time.perf_counter()))
                ld.release(i)

        th = threading.Thread(target=consumer)
        th.start()
        issued = {}
        for i in range(steps):
            ld.step(i)
            issued[i] = time.perf_counter()
        ld.flush()
        th.join(60)
        res["pull_ok"] = ok
        held = {i: t for kind, i, t in log if kind == "held"}
        rel = {i: t for kind, i, t in log if kind == "released"}
        # step i+1 was loaded and gathered while step i was held
        res["overlap"] = sum(1 for i in range(steps - 1) if held[i] < issued[i + 1] < rel[i])
        # step i+2 (same ring buffer) never gathered before step i's release
        res["ring_respected"] = all(issued[i + 2] >= rel[i] for i in range(steps - 2))
        ld.close()
        # (b) callback consumer
        got = []
        ld = ShardedLoader(f"{path}.{r}", window, dev, segment_sz=window // 2, chunk_sz=8192,
                           depth=2, out_ring=3,
                           on_gathered=lambda g: got.append(
                               (g.step, bool(np.array_equal(g.tensor.numpy(), expect(g.step))))))
        ld.run(5)
        res["callback"] = got
        res["delivered"] = ld.report(wall_s=1.0)["delivered_steps_per_rank"]
        ld.close()

        # (c) corruption caught at its step, on every rank
        def corrupt(step, t):
            if r == 2 and step == 2:
                t[777] ^= 0x5A

        ld = ShardedLoader(f"{path}.{r}", window, dev, segment_sz=window // 2, chunk_sz=8192,
                           depth=2, verify_each=True, check_every=1, on_loaded=corrupt)
        caught = None
        try:
            for i in range(5):
                ld.step(i)
            ld.flush()
        except ShardCorruptError as e:
            caught = (e.step, e.failed, ld.last_step)
        res["corrupt"] = caught
        ld.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [4, 8])
def test_fanout_delivers_shards(tmp_path, world):
    """the fan-out delivers every step's gathered shards to a
    consumer (pulled while the next step loads, or via the callback), the
    ring never overwrites a held step, and a corrupted slice is caught at
    its step with every rank agreeing — at 4 ranks and at the 8 of an MI355X
    node (the driver's scaling run)."""
    window = 128 << 10
    path = str(tmp_path / "shard")
    for r in range(world):
        np.random.default_rng(40 + r).integers(0, 256, 4 * window, dtype=np.uint8).tofile(f"{path}.{r}")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_deliver_worker, args=(r, world, port, path, window, q))
          for r in range(world)]
    [p.start() for p in ps]
    try:
        got = dict(q.get(timeout=240) for _ in ps)
    finally:
        [p.join(timeout=60) for p in ps]
        [p.kill() for p in ps if p.is_alive()]
    for r in range(world):
        res = got[r]
        assert isinstance(res, dict), res
        assert res["pull_ok"] == [True] * 6
        assert res["overlap"] >= 3, res
        assert res["ring_respected"]
        assert res["callback"] == [(i, True) for i in range(5)]
        assert res["delivered"] == [5] * world
        assert res["corrupt"] == (2, [2], 2), res["corrupt"]
