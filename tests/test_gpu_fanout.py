"""The fan-out's device path on the one-GPU box: a one-rank
RCCL group with ``force_fan`` runs the side-stream collectives, the ring of
gathered outputs with device events, the consumer stream and the per-step
slice CRCs exactly as each rank of an 8-GPU node does (the multi-rank
schedule itself is covered by the 4-rank gloo tests in
tests/test_parallel_cpu.py)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl1():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    try:
        yield dev
    finally:
        dist.destroy_process_group()


def _file(tmp_path, nbytes, seed=3):
    p = str(tmp_path / "shard.bin")
    data = np.random.default_rng(seed).integers(0, 256, nbytes, dtype=np.uint8)
    data.tofile(p)
    return p, data


def test_device_ring_pull_callback_and_slice_check(tmp_path, rccl1):
    import nvme_strom_amd as S
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.parallel.fanout import ShardCorruptError, ShardedLoader
    S.configure(gpu_emulation=0)
    dev = rccl1
    W = 4 << 20
    path, data = _file(tmp_path, 4 * W)
    want = [S.crc32c_host(data[j * W:(j + 1) * W].tobytes()) for j in range(4)]
    # pull: a consumer stream reads step i's output while step i+1 loads
    cs = torch.cuda.Stream(device=dev)
    got = []
    with ShardedLoader(path, W, dev, segment_sz=1 << 20, depth=2, out_ring=2,
                       verify_each=True, force_fan=True) as ld:
        assert ld.side is not None and ld.fan
        for i in range(6):
            ld.step(i)
            g = ld.gathered(i)
            with torch.cuda.stream(cs):
                g.wait(cs)
                got.append(V.crc32c(g.slice(0)))
            ld.release(i, cs)
        ld.flush()
        rep = ld.report(wall_s=1.0)
        assert ld.verify(5)
    assert got == [want[i % 4] for i in range(6)]
    assert rep["slice_check_ms_per_rank"][0] > 0
    # callback: every step delivered once, on the consumer stream
    seen = []

    def consume(g):
        assert torch.cuda.current_stream(dev) == ld.consumer
        seen.append((g.step, V.crc32c(g.slice(0))))

    with ShardedLoader(path, W, dev, segment_sz=1 << 20, depth=2, out_ring=3,
                       on_gathered=consume, force_fan=True) as ld:
        ld.run(5)
        assert ld.report(wall_s=1.0)["delivered_steps_per_rank"] == [5]
    assert seen == [(i, want[i % 4]) for i in range(5)]

    # a slice corrupted after it landed is caught at its step
    def corrupt(step, t):
        if step == 3:
            t[4097] ^= 0x11

    with ShardedLoader(path, W, dev, segment_sz=1 << 20, depth=2, verify_each=True,
                       check_every=1, on_loaded=corrupt, force_fan=True) as ld:
        with pytest.raises(ShardCorruptError) as e:
            for i in range(6):
                ld.step(i)
        assert e.value.step == 3 and e.value.failed == [0]
