"""Host codecs and checksums (CPU references for the GPU kernels)."""
import struct

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


def test_pg_visibility_frozen_and_all_visible():
    """Frozen rows (xmin COMMITTED|INVALID = 0x0300) are visible; rows with no
    hint bits are visible only on a PD_ALL_VISIBLE page (reference
    pgsql/nvme_strom.c:870-891 takes such pages without per-tuple checks)."""
    vals = np.arange(300, dtype=np.int64)
    # 3 pages of 100; page 0 all-visible (rows unhinted), rows 1,4,7.. frozen
    data = pgpage.build_table(vals, per_page=100, width=8, frozen_every=3,
                              all_visible_every=3, invisible_every=10)
    flags = [int.from_bytes(data[p * 8192 + 10:p * 8192 + 12], "little") for p in range(3)]
    assert flags == [pgpage.PD_ALL_VISIBLE, 0, 0]
    items, status = pgpage.host_scan(data, skip_invisible=True, verify_checksum=True)
    assert status == [0, 0, 0]
    rows = {(it >> 16) * 100 + (it & 0xffff) - 1 for it in items}
    # page 0: every row although none carries a hint bit
    assert all(r in rows for r in range(100))
    # pages 1-2: invisible rows (every 10th) dropped, frozen rows kept
    for r in range(100, 300):
        assert (r in rows) == (r % 10 != 0), r
    frozen = [r for r in range(100, 300) if r % 3 == 1 and r % 10 != 0]
    assert frozen and all(r in rows for r in frozen)
    # the same page without PD_ALL_VISIBLE: unhinted rows are not provably visible
    noflag = bytearray(data)
    noflag[10:12] = b"\0\0"
    items2, _ = pgpage.host_scan(bytes(noflag), skip_invisible=True)
    assert not any((it >> 16) == 0 for it in items2)


def test_pg_tuple_visible_rules():
    V = pgpage.tuple_visible
    assert V(pgpage.HEAP_XMIN_COMMITTED | pgpage.HEAP_XMAX_INVALID, 0)
    assert V(pgpage.HEAP_XMIN_FROZEN | pgpage.HEAP_XMAX_INVALID, 0)
    assert V(pgpage.HEAP_XMIN_COMMITTED | pgpage.HEAP_XMAX_LOCK_ONLY, 0)
    assert not V(pgpage.HEAP_XMIN_INVALID | pgpage.HEAP_XMAX_INVALID, 0)   # aborted
    assert not V(pgpage.HEAP_XMAX_INVALID, 0)                               # xmin unknown
    assert not V(pgpage.HEAP_XMIN_COMMITTED, 0)                             # deleted / unknown xmax
    assert V(0, pgpage.PD_ALL_VISIBLE)


# ---------------------------------------------- block-parallel LZ4 decoder
def _ints(kind, n, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "uniform":          # the config-5 val column: int64 in [0, 1e6)
        return rng.integers(0, 1_000_000, n // 8, dtype=np.int64).tobytes()
    if kind == "sorted":
        return np.arange(n // 8, dtype=np.int64).tobytes()
    return rng.random(n // 8).tobytes()


@pytest.mark.parametrize("threads", [256, 512, "512b"])
@pytest.mark.parametrize("kind", ["random", "text", "runs", "zeros", "uniform", "sorted", "floats"])
@pytest.mark.parametrize("n", [1, 13, 100, 4096, 70000, 300000])
def test_lz4par_raw_block_matches_host(kind, n, threads):
    """Speculative parallel parse + pointer doubling (the GPU kernel's own
    phases, run thread by thread on the CPU, in both builds' geometry) ==
    the serial host decoder."""
    d = (_data(kind, n) if kind in ("random", "text", "runs", "zeros") else _ints(kind, n))[:n]
    c = D.lz4_compress(d)
    st, out, stats = D.lz4par_host(D.LZ4, c, len(d), threads)
    assert st == len(d) and out == d, (st, stats)


@pytest.mark.parametrize("threads", [256, 512, "512b"])
@pytest.mark.parametrize("kind", ["uniform", "sorted", "text", "random"])
def test_lz4par_arrow_frames_from_pyarrow(kind, threads):
    """pyarrow's LZ4 frames (linked 64 KiB blocks: matches reach into the
    previous block) as Arrow IPC buffers, and a stored (-1) buffer."""
    pa = pytest.importorskip("pyarrow")
    d = _ints(kind, 512 << 10, 3) if kind in ("uniform", "sorted") else _data(kind, 512 << 10, 3)
    frame = pa.compress(d, codec="lz4", asbytes=True)
    buf = D.arrow_lz4_buffer(d, frame)
    st, out, stats = D.lz4par_host(D.ARROW_LZ4, buf, len(d), threads)
    assert st == len(d) and out == d, (st, stats)
    raw = b"\xff" * 8 + d[:5000]
    st, out, _ = D.lz4par_host(D.ARROW_LZ4, raw, 5000, threads)
    assert st == 5000 and out == d[:5000]


@pytest.mark.parametrize("threads", [256, 512, "512b"])
def test_lz4par_walkers(threads):
    """The speculative walkers (lz4par.hip NW, WALK_AFTER): dense text —
    whose single chains phase-lock — switches to them in its first window
    and then validates in one scan per window; an int column does not
    switch (64-byte slices); a literal-heavy column (bench kind ``chars``) keeps the serial
    walk.  Every output equals the source."""
    pytest.importorskip("pyarrow")
    from nvme_strom_amd.tools.lz4par_bench import frames
    for kind in ("text", "val", "chars"):
        raws, bufs = frames(kind, 1)
        st, out, stats = D.lz4par_host(D.ARROW_LZ4, bufs[0], len(raws[0]), threads)
        assert st == len(raws[0]) and out == raws[0], (kind, stats)
        if kind == "text":
            assert stats["walk_windows"] == stats["windows"]
            assert stats["rounds"] < 2 * stats["windows"] + 24, stats   # + the first window's
        elif kind == "val":
            if threads == 256:          # 32-byte slices: some windows switch
                assert stats["walk_windows"] == 0
        else:
            assert stats["serial_windows"] == stats["windows"]


@pytest.mark.parametrize("threads", [256, 512, "512b"])
def test_snappy_walkers(threads):
    """Snappy streams walk from their first window (lz4par.hip SN_WALK):
    sorted ids, whose settled-prefix validation re-walked ~3 slices a
    window, validate in one scan per window with no re-parse."""
    pytest.importorskip("pyarrow")
    from nvme_strom_amd.tools.lz4par_bench import frames
    for kind in ("ids", "val", "text"):
        raws, bufs = frames(kind, 2, codec="snappy")
        for raw, buf in zip(raws, bufs):
            st, out, stats = D.lz4par_host(D.SNAPPY, buf, len(raw), threads)
            assert st == len(raw) and out == raw, (kind, stats)
            assert stats["walk_windows"] == stats["windows"]
            assert stats["rounds"] <= stats["windows"] + 4, (kind, stats)


@pytest.mark.parametrize("threads", [256, 512, "512b"])
@pytest.mark.parametrize("kind", ["uniform", "sorted", "floats", "text", "random", "zeros", "runs"])
def test_snappy_block_parallel_from_pyarrow(kind, threads):
    """Raw snappy buffers from pyarrow (and our host compressor) decode
    through the block-parallel phases with snappy's element grammar
    (lz4par.hip SN=true), with the preamble length checked."""
    pa = pytest.importorskip("pyarrow")
    d = (_ints(kind, 512 << 10, 13) if kind in ("uniform", "sorted", "floats")
         else _data(kind, 512 << 10, 13))
    for c in (pa.compress(d, codec="snappy", asbytes=True), D.snappy_compress(d)):
        st, out, stats = D.lz4par_host(D.SNAPPY, c, len(d), threads)
        assert st == len(d) and out == d, (st, stats)
    for n in (0, 1, 2, 63, 64, 65, 70000):
        c = pa.compress(d[:n], codec="snappy", asbytes=True)
        st, out, _ = D.lz4par_host(D.SNAPPY, c, max(n, 1), threads)
        assert st == n and out[:n] == d[:n]


def test_snappy_block_parallel_errors():
    pa = pytest.importorskip("pyarrow")
    d = _data("text", 100000, 5)
    c = pa.compress(d, codec="snappy", asbytes=True)
    assert D.lz4par_host(D.SNAPPY, c, len(d) - 1)[0] == -2      # preamble > capacity
    assert D.lz4par_host(D.SNAPPY, c[: len(c) // 2], len(d))[0] < 0
    # a stream that decodes to fewer bytes than its preamble claims
    short = bytes([0x90, 0x03]) + c[3:]
    assert D.lz4par_host(D.SNAPPY, short, 1 << 20)[0] < 0
    rng = np.random.default_rng(9)
    for _ in range(30):
        g = rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8).tobytes()
        assert D.lz4par_host(D.SNAPPY, g, 1 << 16)[0] <= 1 << 16


def test_lz4par_frames_and_errors():
    d = _data("text", 200000, 5)
    f = D.lz4_frame_compress(d, 64 << 10)
    info = D.parse_lz4_frame_header(f)
    st, out, _ = D.lz4par_host(D.LZ4_FRAME, f[info.data_offset:], len(d))
    assert st == len(d) and out == d
    # random data: stored (uncompressed) blocks
    r = _data("random", 150000, 6)
    f = D.lz4_frame_compress(r, 64 << 10)
    info = D.parse_lz4_frame_header(f)
    st, out, _ = D.lz4par_host(D.LZ4_FRAME, f[info.data_offset:], len(r))
    assert st == len(r) and out == r
    # overflow, truncation and garbage are reported, never crash
    c = D.lz4_compress(d)
    assert D.lz4par_host(D.LZ4, c, len(d) - 1)[0] == -2
    assert D.lz4par_host(D.LZ4, c[: len(c) // 2], len(d))[0] < 0
    rng = np.random.default_rng(9)
    for _ in range(20):
        g = rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8).tobytes()
        assert D.lz4par_host(D.LZ4, g, 1 << 16)[0] <= 1 << 16


# ------------------------------------------------------------------- zstd
def _zstd_payloads():
    rng = np.random.default_rng(11)
    return {
        "zeros": bytes(300000),
        "random": _data("random", 200000, 1),
        "text": _data("text", 330000, 2),
        "runs": _data("runs", 250000, 3),
        "uniform": _ints("uniform", 512 << 10, 4),
        "sorted": _ints("sorted", 512 << 10, 5),
        "floats": _ints("floats", 512 << 10, 6),
        "tiny": b"abc",
        "empty": b"",
        "mixed": b"".join([_data("text", 5000, 7), _data("random", 3000, 8)] * 40),
        "big": _data("text", 1 << 20, 9) + _ints("uniform", 1 << 20, 10),
    }


@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19])
def test_zstd_host_matches_pyarrow(level):
    """The zstd kernel's phases (run lane by lane on the CPU) decode
    pyarrow's zstd frames at fast, default and high levels: raw / RLE /
    compressed blocks, raw / RLE / Huffman literals (1 and 4 streams, FSE
    and direct weights, treeless), predefined / RLE / FSE / repeat sequence
    tables, repeat offsets, multi-block frames."""
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("zstd", compression_level=level)
    for kind, d in _zstd_payloads().items():
        st, out = D.zstd_host(D.ZSTD, codec.compress(d, asbytes=True), len(d))
        assert st == len(d) and out == d, (kind, st)


@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19])
@pytest.mark.parametrize("nw", [2, 4, 8])
def test_zstd_host_frame_parallel_matches_pyarrow(level, nw):
    """The frame-parallel decoder's phases (blocks of a frame decoded on
    nw waves, sequences with symbolic repeat offsets, executed in block
    order) decode the same frames; groups really run blocks ahead (a
    treeless / repeat-table block starts a group of its own)."""
    pa = pytest.importorskip("pyarrow")
    from nvme_strom_amd import _native as N
    codec = pa.Codec("zstd", compression_level=level)
    ahead = 0
    stats = np.zeros(2, np.uint32)
    for kind, d in _zstd_payloads().items():
        st, out = D.zstd_host(D.ZSTD, codec.compress(d, asbytes=True), len(d), fp=nw)
        assert st == len(d) and out == d, (kind, st)
        N.lib().strom_zstd_host_fp_stats(stats.ctypes.data)
        ahead += int(stats[1])
    assert ahead > 0


def test_zstd_host_frame_parallel_arrow_and_errors():
    pa = pytest.importorskip("pyarrow")
    d = _ints("uniform", 512 << 10, 12)
    frame = pa.Codec("zstd").compress(d, asbytes=True)
    assert D.zstd_host(D.ARROW_ZSTD, D.arrow_zstd_buffer(d, frame), len(d), fp=4) == (len(d), d)
    raw = b"\xff" * 8 + d[:5000]
    assert D.zstd_host(D.ARROW_ZSTD, raw, 5000, fp=4) == (5000, d[:5000])
    assert D.zstd_host(D.ZSTD, frame, len(d) - 1, fp=4)[0] == -2          # overflow
    assert D.zstd_host(D.ZSTD, frame[: len(frame) // 2], len(d), fp=4)[0] < 0
    a, b = _data("text", 300000, 13), _data("runs", 290000, 14)
    skip = struct.pack("<II", 0x184D2A53, 5) + b"12345"
    two = pa.Codec("zstd").compress(a, asbytes=True) + skip + \
        pa.Codec("zstd", compression_level=7).compress(b, asbytes=True)
    assert D.zstd_host(D.ZSTD, two, len(a) + len(b), fp=4) == (len(a) + len(b), a + b)
    # mutants: bounded status, same as the serial decoder's contract
    rng = np.random.default_rng(16)
    base = bytearray(frame)
    for i in range(300):
        m = bytearray(base)
        for _ in range(int(rng.integers(1, 6))):
            m[int(rng.integers(4, len(m)))] = int(rng.integers(0, 256))
        st, out = D.zstd_host(D.ZSTD, bytes(m), len(d), fp=4)
        assert st <= len(d)


def test_zstd_arrow_buffers_and_frames():
    pa = pytest.importorskip("pyarrow")
    d = _ints("uniform", 512 << 10, 12)
    frame = pa.Codec("zstd").compress(d, asbytes=True)
    buf = D.arrow_zstd_buffer(d, frame)
    assert D.zstd_host(D.ARROW_ZSTD, buf, len(d)) == (len(d), d)
    # stored (-1) buffer, wrong length prefix
    raw = b"\xff" * 8 + d[:5000]
    assert D.zstd_host(D.ARROW_ZSTD, raw, 5000) == (5000, d[:5000])
    bad = struct.pack("<q", len(d) - 8) + frame
    assert D.zstd_host(D.ARROW_ZSTD, bad, len(d))[0] < 0
    # two frames with a skippable frame between them
    a, b = _data("text", 70000, 13), _data("runs", 90000, 14)
    skip = struct.pack("<II", 0x184D2A53, 5) + b"12345"
    two = pa.Codec("zstd").compress(a, asbytes=True) + skip + pa.Codec("zstd", compression_level=7).compress(b, asbytes=True)
    assert D.zstd_host(D.ZSTD, two, len(a) + len(b)) == (len(a) + len(b), a + b)


def test_zstd_errors_are_bounded():
    pa = pytest.importorskip("pyarrow")
    d = _data("text", 200000, 15)
    c = pa.Codec("zstd").compress(d, asbytes=True)
    assert D.zstd_host(D.ZSTD, c, len(d) - 1)[0] == -2          # overflow
    assert D.zstd_host(D.ZSTD, c[: len(c) // 2], len(d))[0] < 0  # truncated
    # a dictionary id is refused (Arrow writes none)
    hdr = bytes([0x28, 0xB5, 0x2F, 0xFD, 0x21, 0x07]) + b"\x01\x00\x00"
    assert D.zstd_host(D.ZSTD, hdr, 100)[0] == -4
    # mutated frames never read or write out of range (the GPU kernel
    # runs the same checks); ASan coverage: csrc/tests/zstd_fuzz.cc
    rng = np.random.default_rng(16)
    base = bytearray(c)
    for i in range(200):
        m = bytearray(base)
        for _ in range(int(rng.integers(1, 6))):
            m[int(rng.integers(4, len(m)))] = int(rng.integers(0, 256))
        st, out = D.zstd_host(D.ZSTD, bytes(m), len(d))
        assert st <= len(d)


def test_lz4par_fuzz_asan(tmp_path):
    """Random edits / truncations of pyarrow LZ4 frames and snappy buffers
    through the block-parallel decoder's phases built host-only with ASan +
    UBSan (csrc/tests/lz4par_fuzz.cc): the text seeds run on the walkers
    (LZ4 switches to them, snappy starts on them); seeds decode exactly,
    mutants end in a clean status within the capacity."""
    pa = pytest.importorskip("pyarrow")
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "build/lz4par_fuzz"], cwd=root, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    args = []
    seeds = [_data("text", 150000, 2), _ints("uniform", 160000, 1), _ints("sorted", 120000, 3)]
    for i, d in enumerate(seeds):
        for codec, enc in ((D.ARROW_LZ4, lambda x: D.arrow_lz4_buffer(
                x, pa.compress(x, codec="lz4", asbytes=True))),
                           (D.SNAPPY, lambda x: pa.compress(x, codec="snappy", asbytes=True))):
            (tmp_path / f"{i}_{codec}.bin").write_bytes(enc(d))
            (tmp_path / f"{i}_{codec}.raw").write_bytes(d)
            args += [str(codec), str(tmp_path / f"{i}_{codec}.bin"),
                     str(tmp_path / f"{i}_{codec}.raw")]
    r = subprocess.run([os.path.join(root, "build", "lz4par_fuzz"), "150"] + args,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "6 seeds ok" in r.stdout


def test_zstd_fuzz_asan(tmp_path):
    """8k random edits / truncations of real zstd frames through the
    decoder's phases built host-only with ASan + UBSan
    (csrc/tests/zstd_fuzz.cc): seeds decode exactly, mutants end in a
    clean status, never an out-of-range access."""
    pa = pytest.importorskip("pyarrow")
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "build/zstd_fuzz"], cwd=root, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    args = []
    seeds = [(1, _ints("uniform", 160000, 1)), (3, _data("text", 150000, 2)),
             (19, _ints("sorted", 240000, 3)), (-3, _ints("floats", 40000, 4))]
    for i, (lvl, d) in enumerate(seeds):
        z = pa.Codec("zstd", compression_level=lvl).compress(d, asbytes=True)
        (tmp_path / f"{i}.zst").write_bytes(z)
        (tmp_path / f"{i}.raw").write_bytes(d)
        args += [str(tmp_path / f"{i}.zst"), str(tmp_path / f"{i}.raw")]
    r = subprocess.run([os.path.join(root, "build", "zstd_fuzz"), "2000"] + args,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "4 seeds ok" in r.stdout


def _with_checksum(frame: bytes, data: bytes) -> bytes:
    """A pyarrow zstd frame re-marked with the content-checksum flag and the
    XXH64 (seed 0) low 32 bits appended, as the zstd CLI writes frames."""
    xxhash = pytest.importorskip("xxhash")
    f = bytearray(frame)
    f[4] |= 0x04
    return bytes(f) + struct.pack("<I", xxhash.xxh64_intdigest(data, 0) & 0xFFFFFFFF)


@pytest.mark.parametrize("n", [0, 5, 31, 32, 33, 100, 4096 + 7, 300000])
def test_zstd_content_checksum(n):
    """Frames carrying a content checksum decode and verify (XXH64 over the
    frame's output: the four stripe accumulators on lanes 0..3 + the tail);
    a wrong checksum is reported as -5."""
    pa = pytest.importorskip("pyarrow")
    d = _data("text", n, 17)
    z = _with_checksum(pa.Codec("zstd").compress(d, asbytes=True), d)
    assert D.zstd_host(D.ZSTD, z, len(d)) == (len(d), d)
    bad = z[:-1] + bytes([z[-1] ^ 0x01])
    assert D.zstd_host(D.ZSTD, bad, len(d))[0] == -5


# ------------------------------------------------------- zstd lane-parallel
@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19])
def test_zstd_host_lane_parallel_matches_pyarrow(level):
    """The lane-parallel decoder's phases (walk per stream; entropy stages
    of LPB blocks per wave, a lane per literal stream / sequence bitstream,
    literals packed at the output's tail; executions in block order) over
    every payload at once: each decodes exactly, and on the LP path itself
    (no serial fallback) — raw / RLE / compressed blocks, treeless
    literals, repeat-mode tables and symbolic repeat offsets included."""
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("zstd", compression_level=level)
    pl = _zstd_payloads()
    bufs = [codec.compress(d, asbytes=True) for d in pl.values()]
    st, outs, taken = D.zstd_host_lp(D.ZSTD, bufs, [len(d) for d in pl.values()])
    for (kind, d), s, o in zip(pl.items(), st, outs):
        assert s == len(d) and o == d, (kind, s)
    assert taken == len(bufs)


def test_zstd_host_lane_parallel_arrow_fallbacks_and_errors():
    """Streams the walk refuses (a stored Arrow buffer, several frames, a
    dictionary) and broken ones go to the serial decoder inside the exec
    phase: the statuses and outputs equal the serial decoder's, mutants
    included; an entry pool too small for every stream sends the rest to
    the serial decoder, still exact."""
    pa = pytest.importorskip("pyarrow")
    d = _ints("uniform", 512 << 10, 12)
    frame = pa.Codec("zstd").compress(d, asbytes=True)
    a, b = _data("text", 70000, 13), _data("runs", 90000, 14)
    skip = struct.pack("<II", 0x184D2A53, 5) + b"12345"
    two = pa.Codec("zstd").compress(a, asbytes=True) + skip + \
        pa.Codec("zstd", compression_level=7).compress(b, asbytes=True)
    st, outs, taken = D.zstd_host_lp(D.ARROW_ZSTD, [D.arrow_zstd_buffer(d, frame),
                                                    b"\xff" * 8 + d[:5000]], [len(d), 5000])
    assert st == [len(d), 5000] and outs == [d, d[:5000]] and taken == 1
    st, outs, taken = D.zstd_host_lp(D.ZSTD, [two, frame, frame, frame[: len(frame) // 2]],
                                     [len(a) + len(b), len(d), len(d) - 1, len(d)])
    assert st[:3] == [len(a) + len(b), len(d), -2] and outs[:2] == [a + b, d]
    assert st[3] < 0 and taken == 1
    # pool exhaustion: some streams fall back, all exact
    bufs = [frame] * 6
    st, outs, taken = D.zstd_host_lp(D.ZSTD, bufs, [len(d)] * 6, ent_factor=0.6)
    assert st == [len(d)] * 6 and all(o == d for o in outs) and 0 < taken < 6
    # mutants: the LP statuses / outputs are the serial decoder's
    rng = np.random.default_rng(21)
    for src, cap in ((frame, len(d)), (pa.Codec("zstd", compression_level=3).compress(
            _data("text", 200000, 15), asbytes=True), 200000)):
        muts = []
        for _ in range(120):
            m = bytearray(src)
            for _ in range(int(rng.integers(1, 6))):
                m[int(rng.integers(4, len(m)))] = int(rng.integers(0, 256))
            muts.append(bytes(m))
        st, outs, _ = D.zstd_host_lp(D.ZSTD, muts, [cap] * len(muts))
        for m, s, o in zip(muts, st, outs):
            ss, so = D.zstd_host(D.ZSTD, m, cap)
            assert (s, o) == (ss, so)
