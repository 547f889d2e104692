"""Statistics export: the shared-memory counters are visible to an external
viewer (strom_stat / utils.stat) while the engine runs."""
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shm_export_matches_ioctl(strom, rand_file):
    from nvme_strom_amd.utils import stat
    path, _ = rand_file(32 * 8192)
    fd = os.open(path, os.O_RDONLY)
    try:
        with strom.alloc_dma_buffer(32 * 8192) as buf:
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(32, dtype=np.uint32), 8192)
            strom.memcpy_wait(r.dma_task_id)
    finally:
        os.close(fd)
    ex = stat.read_exports(os.getpid())
    assert os.getpid() in ex
    mine = ex[os.getpid()]
    info = strom.stat_info()
    assert mine["nr_ssd2gpu"] == info["nr_ssd2gpu"] > 0
    assert mine["nr_submit_dma"] == info["nr_submit_dma"]
    assert mine["io_ns"].sum() >= 1


def test_strom_stat_binary_reads_export(strom, rand_file):
    tool = os.path.join(ROOT, "nvme_strom_amd", "lib", "strom_stat")
    if not os.path.exists(tool):
        import pytest
        pytest.skip("tools not built")
    strom.stat_info()   # make sure this process exports
    out = subprocess.run([tool, "-p", str(os.getpid())], capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stderr
    assert "ssd2gpu" in out.stdout and "latency(us)" in out.stdout
