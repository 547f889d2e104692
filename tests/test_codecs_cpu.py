"""Host codecs and checksums (CPU references for the GPU kernels)."""
import numpy as np
import pytest

import nvme_strom_amd as S
from nvme_strom_amd.ops import decompress as D
from nvme_strom_amd.utils import pgpage


def _data(kind, n, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "text":
        words = [b"alpha", b"beta", b"gamma", b"delta", b"nvme", b"strom", b"mi355x"]
        out = b" ".join(words[i] for i in rng.integers(0, len(words), n // 5 + 1))
        return out[:n]
    if kind == "runs":
        return b"".join(bytes([rng.integers(0, 4)]) * int(rng.integers(1, 300)) for _ in range(n // 100 + 1))[:n]
    return bytes(n)


def test_crc32c_vectors():
    assert S.crc32c_host(b"") == 0
    assert S.crc32c_host(b"123456789") == 0xE3069283
    assert S.crc32c_host(bytes(32)) == 0x8A9136AA
    # incremental == one-shot
    d = _data("random", 10000)
    assert S.crc32c_host(d[5000:], S.crc32c_host(d[:5000])) == S.crc32c_host(d)


@pytest.mark.parametrize("kind", ["random", "text", "runs", "zeros"])
@pytest.mark.parametrize("n", [0, 1, 13, 4096, 100000])
def test_lz4_roundtrip(kind, n):
    d = _data(kind, n)
    c = D.lz4_compress(d)
    assert D.lz4_decompress(c, n) == d


@pytest.mark.parametrize("kind", ["random", "text", "runs", "zeros"])
@pytest.mark.parametrize("n", [0, 1, 13, 4096, 100000])
def test_snappy_roundtrip(kind, n):
    d = _data(kind, n)
    c = D.snappy_compress(d)
    assert D.snappy_decompress(c, n) == d


def test_codecs_interop_with_pyarrow():
    pa = pytest.importorskip("pyarrow")
    d = _data("text", 200000, 3)
    # pyarrow's snappy / lz4_raw streams decode with our host decoders
    assert D.snappy_decompress(pa.compress(d, codec="snappy", asbytes=True), len(d)) == d
    assert D.lz4_decompress(pa.compress(d, codec="lz4_raw", asbytes=True), len(d)) == d
    # and ours decode with pyarrow's
    assert pa.decompress(D.snappy_compress(d), len(d), codec="snappy", asbytes=True) == d
    assert pa.decompress(D.lz4_compress(d), len(d), codec="lz4_raw", asbytes=True) == d


def test_lz4_frame_header():
    pa = pytest.importorskip("pyarrow")
    fr = pa.compress(_data("text", 300000), codec="lz4", asbytes=True)
    info = D.parse_lz4_frame_header(fr)
    assert info.data_offset >= 7
    ours = D.lz4_frame_compress(_data("text", 300000))
    assert pa.decompress(ours, 300000, codec="lz4", asbytes=True) == _data("text", 300000)


def test_pg_page_builder_and_checksum():
    vals = np.arange(100, dtype=np.int64)
    data = pgpage.build_table(vals, per_page=40, width=8)
    assert len(data) == 3 * 8192
    items, status = pgpage.host_scan(data, verify_checksum=True)
    assert status == [0, 0, 0] and len(items) == 100
    # a flipped byte breaks the checksum of that page only
    bad = bytearray(data)
    bad[8192 + 5000] ^= 0xFF
    _, status = pgpage.host_scan(bytes(bad), verify_checksum=True)
    assert status == [0, 2, 0]
    # filter on the int8 column
    items, _ = pgpage.host_scan(data, attr_off=0, attr_width=8, lo=10, hi=19)
    assert len(items) == 10
