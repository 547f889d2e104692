"""CLI tools: ssd2ram_test on CPU (data check on), strom_test on the GPU."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "nvme_strom_amd", "lib")


def _tool(name):
    p = os.path.join(LIB, name)
    if not os.path.exists(p):
        pytest.skip(f"{name} not built")
    return p


def _env():
    return dict(os.environ, STROM_WORKERS="2")


def test_ssd2ram_test_cli(rand_file):
    path, _ = rand_file(8 << 20)
    out = subprocess.run([_tool("ssd2ram_test"), "-n", "3", "-s", "4", "-c", path],
                         capture_output=True, text=True, timeout=120, env=_env())
    assert out.returncode == 0, out.stdout + out.stderr
    assert "verify: 0 corrupted" in out.stdout
    assert "throughput" in out.stdout


def test_ssd2ram_test_print(rand_file):
    path, _ = rand_file(1 << 20)
    out = subprocess.run([_tool("ssd2ram_test"), "-p", path], capture_output=True, text=True,
                         timeout=60, env=_env())
    assert out.returncode == 0 and "support_dma64: 1" in out.stdout


@pytest.mark.gpu
def test_strom_test_cli_verify(rand_file):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    path, _ = rand_file(48 << 20)
    out = subprocess.run([_tool("strom_test"), "-c", "-n", "3", "-s", "8", path],
                         capture_output=True, text=True, timeout=300, env=_env())
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 corrupted" in out.stdout
    vfs = subprocess.run([_tool("strom_test"), "-f", "-c", "-n", "3", "-s", "8", path],
                         capture_output=True, text=True, timeout=300, env=_env())
    assert vfs.returncode == 0, vfs.stdout + vfs.stderr
    pr = subprocess.run([_tool("strom_test"), "-p", path], capture_output=True, text=True,
                        timeout=120, env=_env())
    assert pr.returncode == 0 and "mapped region" in pr.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("spec", ["100:300", "100:300:256", "13:13"])
def test_strom_test_cli_extents(rand_file, spec):
    """strom_test -e: MEMCPY_SSD2GPU_EXTENTS per segment, every landed extent
    compared with pread of its file range; holes read through with a gap."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    path, _ = rand_file((40 << 20) + 12345)            # a partial last extent
    out = subprocess.run([_tool("strom_test"), "-c", "-n", "3", "-s", "8", "-e", spec, path],
                         capture_output=True, text=True, timeout=300, env=_env())
    assert out.returncode == 0, out.stdout + out.stderr
    assert "SSD2GPU_EXTENTS" in out.stdout and " 0 corrupted" in out.stdout, out.stdout
    ln, stride = (int(v) for v in spec.split(":")[:2])
    amp = float(out.stdout.split("(")[-1].split(" of the")[0]) if "of the" in out.stdout else None
    if spec.count(":") == 2:                           # 200 KiB holes read through
        assert amp is not None and amp > 2.5
    elif ln == stride:
        assert amp is not None and amp < 1.01


def test_block_sweep_cpu(strom, tmp_path):
    """Block-size sweep tool end to end on emulated HBM (small sizes)."""
    from nvme_strom_amd.tools import sweep
    out = tmp_path / "sweep.json"
    rc = sweep.main(["--file-gib", "0.125", "--dir", str(tmp_path), "--blocks", "4K,64K,1M",
                     "--max-gib", "0.0625", "--lat-samples", "20", "--device", "cpu",
                     "--out", str(out)])
    assert rc == 0
    import json
    rows = json.load(open(out))["rows"]
    assert [r["block"] for r in rows] == [4096, 65536, 1 << 20]
    for r in rows:
        assert r["GiBps"] > 0 and r["p50_us"] > 0
        assert r["avg_req_kib"] <= r["block"] / 1024
        assert r["raw_iops"] > 0 and r["raw_GiBps"] > 0
    assert strom.config_get("max_request") == str(1 << 20)   # restored


def test_block_sweep_engine_only_ab_cpu(strom, tmp_path):
    """--engine-only (backend=cache, storage removed) with an interleaved
    A/B of a config key: both arms per size, config restored after."""
    from nvme_strom_amd.tools import sweep
    out = tmp_path / "sweep_cache.json"
    rc = sweep.main(["--file-gib", "0.0625", "--dir", str(tmp_path), "--blocks", "4K,64K",
                     "--max-gib", "0.03125", "--lat-samples", "10", "--device", "cpu",
                     "--engine-only", "--ab", "fixed_bufs", "--out", str(out)])
    assert rc == 0
    import json
    res = json.load(open(out))
    assert res["backend"].startswith("cache") and res["ab"] == "fixed_bufs"
    assert [(r["block"], r["fixed_bufs"]) for r in res["rows"]] == [(4096, 0), (4096, 1),
                                                                     (65536, 0), (65536, 1)]
    assert all(r["GiBps"] > 0 and r["raw_GiBps"] > 0 for r in res["rows"])
    assert strom.config_get("backend") == "uring" and strom.config_get("fixed_bufs") == "1"


def test_raw_read_rate(strom, tmp_path):
    """The storage-ceiling probe reads the requested count and rejects bad shapes."""
    import os
    path = tmp_path / "raw.bin"
    path.write_bytes(os.urandom(4 << 20))
    fd = os.open(path, os.O_RDONLY)
    try:
        for seq in (False, True):
            iops, gib = strom.raw_read_rate(fd, 65536, 300, threads=3, qd=4, sequential=seq)
            assert iops > 0 and abs(gib - iops * 65536 / (1 << 30)) < 1e-6 * max(gib, 1)
        for bad in [dict(block=1000, nreq=10), dict(block=4096, nreq=0),
                    dict(block=8 << 20, nreq=10)]:
            with pytest.raises(strom.StromError):
                strom.raw_read_rate(fd, bad["block"], bad["nreq"])
    finally:
        os.close(fd)


def test_raw_read_list(strom, tmp_path):
    """The request-list comparator reads exactly the listed bytes (a read at
    the end comes back short and counts what it read) and rejects unaligned
    or empty requests."""
    import os
    import numpy as np
    path = tmp_path / "rawl.bin"
    size = (4 << 20) + 1000
    path.write_bytes(os.urandom(size))
    fd = os.open(path, os.O_RDONLY)
    try:
        offs = np.arange(0, 4 << 20, 3 << 16, dtype=np.uint64)      # gaps between 64 KiB reads
        lens = np.full(len(offs), 65536, dtype=np.uint32)
        iops, gib = strom.raw_read_list(fd, offs, lens, threads=3, qd=4)
        assert iops > 0 and abs(gib - iops * 65536 / (1 << 30)) < 1e-6 * max(gib, 1)
        # the last page: 1000 bytes of a 4 KiB request
        iops, gib = strom.raw_read_list(fd, [4 << 20], [4096], threads=2, qd=2)
        assert abs(gib - iops * 1000 / (1 << 30)) < 1e-6 * max(gib, 1)
        for o, n in [([100], [4096]), ([0], [0]), ([0], [1000])]:
            with pytest.raises(strom.StromError):
                strom.raw_read_list(fd, o, n)
        with pytest.raises(ValueError):
            strom.raw_read_list(fd, [0, 4096], [4096])
        with pytest.raises(strom.StromError):           # 256 x 64 MiB of buffers per ring
            strom.raw_read_list(fd, [0], [64 << 20], qd=256)
    finally:
        os.close(fd)
