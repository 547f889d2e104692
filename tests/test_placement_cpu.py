"""Multi-GPU readiness on the CPU: PCIe affinity from a fake sysfs tree,
per-device reader-pool sizing across 4 gloo ranks, and a read failure on
one rank surfacing on every rank (no hang in the next collective).

The reference is single-GPU; these are the placement
and failure rules of the MI355X one-process-per-GPU design.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nvme_strom_amd.utils import topology as T


def _dev(root, chain, vendor="0x1002", cls="0x038000", numa=0):
    """Create /sys/devices/<chain...> and the /sys/bus/pci/devices link."""
    d = os.path.join(root, "devices", *chain)
    os.makedirs(d, exist_ok=True)
    for name, val in (("vendor", vendor), ("class", cls), ("numa_node", str(numa))):
        with open(os.path.join(d, name), "w") as f:
            f.write(val + "\n")
    link = os.path.join(root, "bus", "pci", "devices", chain[-1])
    os.makedirs(os.path.dirname(link), exist_ok=True)
    os.symlink(d, link)
    return d


def _nvme(root, name, chain, numa=0):
    d = _dev(root, chain, vendor="0x144d", cls="0x010802", numa=numa)
    c = os.path.join(root, "class", "nvme", name)
    os.makedirs(c, exist_ok=True)
    os.symlink(d, os.path.join(c, "device"))


@pytest.fixture
def fake_sysfs(tmp_path):
    r = str(tmp_path / "sys")
    h0, h1 = "pci0000:00", "pci0000:80"
    # GPU A behind a switch on root port 00:01.0; nvme0 on the same switch,
    # nvme1 on another root port of the same host bridge
    _dev(r, [h0, "0000:00:01.0", "0000:01:00.0", "0000:02:00.0", "0000:03:00.0"])
    _nvme(r, "nvme0", [h0, "0000:00:01.0", "0000:01:00.0", "0000:02:01.0", "0000:04:00.0"])
    _nvme(r, "nvme1", [h0, "0000:00:03.0", "0000:05:00.0"])
    # GPU B on the other socket; nvme2 directly on its root port's host
    # bridge, nvme3 on a third host bridge of the same node
    _dev(r, [h1, "0000:80:01.0", "0000:81:00.0"], numa=1)
    _nvme(r, "nvme2", [h1, "0000:80:01.0", "0000:81:00.1"], numa=1)
    _nvme(r, "nvme3", ["pci0000:c0", "0000:c0:01.0", "0000:c1:00.0"], numa=1)
    return r


def test_pci_chain_and_affinity(fake_sysfs):
    s = fake_sysfs
    assert T.pci_chain("0000:03:00.0", s) == ["pci0000:00", "0000:00:01.0", "0000:01:00.0",
                                              "0000:02:00.0", "0000:03:00.0"]
    assert T.pci_chain("0000:ff:00.0", s) == []
    assert T.affinity("0000:03:00.0", "0000:04:00.0", s) == "same-switch"
    assert T.affinity("0000:03:00.0", "0000:05:00.0", s) == "same-host-bridge"
    assert T.affinity("0000:81:00.0", "0000:81:00.1", s) == "same-root-port"
    assert T.affinity("0000:81:00.0", "0000:c1:00.0", s) == "same-numa"
    assert T.affinity("0000:03:00.0", "0000:c1:00.0", s) == "cross-numa"
    assert T.affinity("0000:03:00.0", "0000:ee:00.0", s) == "unknown"


def test_rank_controllers_per_gpu(fake_sysfs):
    s = fake_sysfs
    assert T.amd_gpus(s) == ["0000:03:00.0", "0000:81:00.0"]
    assert T.nvme_controllers(s) == {"nvme0": "0000:04:00.0", "nvme1": "0000:05:00.0",
                                     "nvme2": "0000:81:00.1", "nvme3": "0000:c1:00.0"}
    a = [r["ctrl"] for r in T.rank_controllers("0000:03:00.0", s)]
    b = [r["ctrl"] for r in T.rank_controllers("0000:81:00.0", s)]
    assert a == ["nvme0", "nvme1", "nvme2", "nvme3"]
    assert b == ["nvme2", "nvme3", "nvme0", "nvme1"]


def test_file_topology_native(tmp_path):
    p = tmp_path / "f.bin"
    p.write_bytes(b"x" * 8192)
    t = T.file_topology(str(p))
    st = os.stat(p)
    assert t["dev"] == f"{os.major(st.st_dev)}:{os.minor(st.st_dev)}"
    assert t["fs"]
    if t["disk"]:
        assert t["members"] and t["members"][0]["disk"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, window, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        os.environ.pop("STROM_WORKERS", None)
        import torch.distributed as dist
        import nvme_strom_amd as S
        from nvme_strom_amd.parallel import ShardedLoader, ShardLoadError, init_distributed, placement
        S.configure(gpu_emulation=1, workers=4)
        r, w, dev = init_distributed("gloo")
        out = {}
        # every rank's shard lives on the same device here: 4 sharers
        p = placement.plan_io(f"{path}.{r}")
        out["same"] = (p["sharers"], p["workers"], p["distinct_devices"])
        # two devices, two ranks each (identities faked: one SSD per pair)
        real = placement.device_identity
        placement.device_identity = lambda path: (f"h:{'A' if r < 2 else 'B'}", real(path)[1])
        p = placement.plan_io(f"{path}.{r}")
        placement.device_identity = real
        out["split"] = (p["sharers"], p["workers"], p["distinct_devices"])
        assert S.config_get("workers") == "2"
        # one shard file per rank (as on the GPU node): no other rank's
        # buffered reads can pull rank 2's pages into the page cache
        mine = f"{path}.{r}"
        ld = ShardedLoader(mine, window, dev, segment_sz=window // 4, chunk_sz=8192, depth=2)
        ld.step(0)
        ld.flush()
        if r == 2:
            fd = os.open(mine, os.O_RDONLY)
            S.evict_file(fd)                        # storage reads, not page-cache copies
            os.close(fd)
            S.fault_inject(fail_at=1)               # first storage request of step 1
        # no per-step host sync: the failure surfaces at the next check
        # (every K steps or flush), on every rank, with the failed step
        try:
            ld.step(1)
            out["raised_in_step"] = True
            ld.flush()
            out["raised"] = None
        except ShardLoadError as e:
            out["raised"] = (e.step, e.failed, e.cause is not None)
        S.fault_inject(0)
        ld.step(2)                                  # the group carries on after
        ld.flush()
        exp = np.concatenate([np.fromfile(f"{path}.{k}", dtype=np.uint8)[:window]
                              for k in range(w)])
        out["after_ok"] = bool(np.array_equal(ld.out.numpy(), exp))
        ld.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_four_rank_placement_and_failure_consensus(tmp_path):
    world, window = 4, 256 << 10
    path = str(tmp_path / "shard")
    for r in range(world):
        np.random.default_rng(r).integers(0, 256, 2 * window, dtype=np.uint8).tofile(f"{path}.{r}")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, path, window, q)) for r in range(world)]
    [p.start() for p in ps]
    try:
        got = dict(q.get(timeout=180) for _ in ps)
    finally:
        [p.join(timeout=60) for p in ps]
        [p.kill() for p in ps if p.is_alive()]
    for r in range(world):
        assert isinstance(got[r], dict), got[r]
        assert got[r]["same"] == (4, 1, 1)
        assert got[r]["split"] == (2, 2, 2)
        # rank 2's read error reaches every rank, with its cause only there
        assert got[r]["raised"] == (1, [2], r == 2)
        assert got[r]["raised_in_step"]             # step itself did not block/raise
        assert got[r]["after_ok"]
