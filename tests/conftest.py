import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    lib = os.path.join(ROOT, "nvme_strom_amd", "lib", "libstrom.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", ROOT, "-j8", "nvme_strom_amd/lib/libstrom.so"], check=True)


_ensure_built()


@pytest.fixture
def strom():
    import nvme_strom_amd as S
    S.configure(gpu_emulation=1, backend="uring", max_request=1 << 20, pgcache_probe=1,
                strict=0, direct_io=1, workers=4)
    S.fault_inject(0)
    yield S
    S.fault_inject(0)


def make_file(path, nbytes, seed=0, evict=True):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, size=nbytes, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(data.tobytes())
        f.flush()
        os.fsync(f.fileno())
    if evict:
        fd = os.open(path, os.O_RDONLY)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        os.close(fd)
    return data


@pytest.fixture
def rand_file(tmp_path):
    def _mk(nbytes, seed=0, evict=True, name="data.bin"):
        p = str(tmp_path / name)
        return p, make_file(p, nbytes, seed, evict)
    return _mk
