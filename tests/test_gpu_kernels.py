"""GPU kernel numerics vs host references: heap scan, LZ4/snappy, column filter."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def _t(b, dev):
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).to(dev)


# ------------------------------------------------------------------ heap scan
def test_heap_scan_matches_host(dev):
    from nvme_strom_amd.ops.heapscan import heap_scan
    from nvme_strom_amd.utils import pgpage
    rng = np.random.default_rng(0)
    vals = rng.integers(-1000, 1000, 5000).astype(np.int64)
    data = bytearray(pgpage.build_table(vals, per_page=150, width=8, invisible_every=7))
    npages = len(data) // 8192
    data[3 * 8192 + 6000] ^= 0x5A                      # corrupt page 3 payload
    data[5 * 8192:6 * 8192] = bytes(8192)              # page 5 is new/empty
    data = bytes(data)
    t = _t(data, dev)
    for kw in [dict(), dict(skip_invisible=True), dict(verify_checksum=True),
               dict(skip_invisible=True, verify_checksum=True, attr_off=0, attr_width=8,
                    lo=-10, hi=250)]:
        r = heap_scan(t, **kw)
        ref_items, ref_status = pgpage.host_scan(data, **kw)
        assert list(r.sorted_items()) == ref_items, kw
        assert list(r.page_status.cpu().numpy()) == ref_status, kw
    assert npages > 6


def test_heap_scan_frozen_and_all_visible(dev):
    """Frozen rows and PD_ALL_VISIBLE pages (rows without hint bits) are kept
    by skip_invisible, like the host reference (frozen rows were
    dropped)."""
    from nvme_strom_amd.ops.heapscan import heap_scan
    from nvme_strom_amd.utils import pgpage
    vals = np.arange(6000, dtype=np.int64)
    data = pgpage.build_table(vals, per_page=150, width=8, frozen_every=4, all_visible_every=5,
                              invisible_every=11)
    t = _t(data, dev)
    for kw in [dict(skip_invisible=True), dict(skip_invisible=True, verify_checksum=True,
                                               attr_off=0, attr_width=8, lo=100, hi=4000)]:
        r = heap_scan(t, **kw)
        ref_items, ref_status = pgpage.host_scan(data, **kw)
        assert list(r.sorted_items()) == ref_items, kw
        assert list(r.page_status.cpu().numpy()) == ref_status, kw
    r = heap_scan(t, skip_invisible=True)
    assert r.count == 6000 - len([i for i in range(6000) if i % 11 == 0 and (i // 150) % 5])


@pytest.mark.parametrize("page_sz", [4096, 16384, 32768])
def test_heap_scan_other_page_sizes(dev, page_sz):
    from nvme_strom_amd.ops.heapscan import heap_scan
    from nvme_strom_amd.utils import pgpage
    vals = np.arange(20000, dtype=np.int64) - 7000
    per = page_sz // 48
    data = pgpage.build_table(vals, per_page=per, width=8, page_sz=page_sz, invisible_every=13,
                              frozen_every=6)
    kw = dict(page_sz=page_sz, skip_invisible=True, verify_checksum=True, attr_off=0,
              attr_width=8, lo=-50, hi=9000)
    r = heap_scan(_t(data, dev), **kw)
    ref_items, ref_status = pgpage.host_scan(data, **kw)
    assert list(r.sorted_items()) == ref_items
    assert list(r.page_status.cpu().numpy()) == ref_status


def test_heap_scan_int4_column(dev):
    from nvme_strom_amd.ops.heapscan import heap_scan
    from nvme_strom_amd.utils import pgpage
    vals = np.arange(3000, dtype=np.int64) - 1500
    data = pgpage.build_table(vals, per_page=200, width=4)
    r = heap_scan(_t(data, dev), attr_off=0, attr_width=4, lo=0, hi=99)
    assert r.count == 100


# ---------------------------------------------------------------- decompress
def _payloads():
    rng = np.random.default_rng(1)
    words = [b"select", b"from", b"where", b"nvme", b"strom", b"gpu", b"hbm", b"mi355x"]
    text = b" ".join(words[i] for i in rng.integers(0, len(words), 60000))
    runs = b"".join(bytes([int(rng.integers(0, 3))]) * int(rng.integers(1, 500)) for _ in range(800))
    rand = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    ints = np.cumsum(rng.integers(0, 5, 50000)).astype(np.int64).tobytes()
    # matches farther than the 8 KiB LDS ring (read back from HBM output),
    # and a far match overlapping itself (distance 9000 < length)
    r1, r2 = (rng.integers(0, 256, 20000, dtype=np.uint8).tobytes() for _ in range(2))
    far = r1 + r2 + r1[:5000] + r2[3000:9000] + r1
    r3 = rng.integers(0, 256, 9000, dtype=np.uint8).tobytes()
    far_overlap = r3 * 5
    # the config-5 column: int64 uniform in [0, 1e6) — short matches, a
    # quarter of them past 2 KiB (far matches taken in the fast step)
    uni = rng.integers(0, 1_000_000, 40000).astype(np.int64).tobytes()
    return [text, runs, rand, ints, b"x", b"", bytes(200000), far, far_overlap, uni]


# the zstd decoder the zmode fixture selected for _run: None (library
# choice / fp_mode), or D.ZSTD_LP (the lane-parallel kernels)
_ZSTD_ROUTE = {"mode": None}


def _run_lp(codec, streams, sizes, dev):
    """The LP decoder's kernels (walk / lit / seq / exec / serial) through
    decompress_async(zstd_mode=ZSTD_LP) on a stream of their own, and the
    launch's counters: the streams the LP path decoded must equal the host
    twin's (strom_zstd_host_lp) — a silent fallback of every stream to the
    serial decoder fails here."""
    from nvme_strom_amd import _native as N
    from nvme_strom_amd.ops import decompress as D
    from nvme_strom_amd.ops._util import stream_handle
    src = b"".join(streams)
    offs = np.cumsum([0] + [len(s) for s in streams])[:-1]
    doffs = np.cumsum([0] + list(sizes))[:-1]
    descs = D.make_descs([(int(o), len(s), int(do), n) for o, s, do, n in zip(offs, streams, doffs, sizes)])
    dst = torch.zeros(max(1, sum(sizes)), dtype=torch.uint8, device=dev)
    d_src = _t(src + b"\0", dev)
    d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
    status = torch.empty(len(streams), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    D.decompress_async(codec, d_src, dst, d_desc, status, stream=s, zstd_mode=D.ZSTD_LP)
    cnt = np.zeros(4, np.uint64)
    assert N.lib().strom_zstd_lp_last(stream_handle(s), cnt.ctypes.data) == 0
    st = status.cpu().numpy()
    hst, _, taken = D.zstd_host_lp(codec, list(streams), list(sizes))
    assert int(cnt[1]) == taken, (int(cnt[1]), taken)
    assert st.tolist() == hst
    out = dst.cpu().numpy().tobytes()
    return st, [out[int(do):int(do) + n] for do, n in zip(doffs, sizes)]


def _run(codec, streams, sizes, dev):
    from nvme_strom_amd.ops import decompress as D
    if _ZSTD_ROUTE["mode"] == D.ZSTD_LP and codec in (D.ZSTD, D.ARROW_ZSTD):
        return _run_lp(codec, streams, sizes, dev)
    src = b"".join(streams)
    offs = np.cumsum([0] + [len(s) for s in streams])[:-1]
    doffs = np.cumsum([0] + list(sizes))[:-1]
    descs = D.make_descs([(int(o), len(s), int(do), n) for o, s, do, n in zip(offs, streams, doffs, sizes)])
    dst = torch.zeros(max(1, sum(sizes)), dtype=torch.uint8, device=dev)
    st = D.decompress(codec, _t(src + b"\0", dev), dst, descs)
    out = dst.cpu().numpy().tobytes()
    return st, [out[int(do):int(do) + n] for do, n in zip(doffs, sizes)]


@pytest.mark.parametrize("codec", ["lz4", "snappy"])
def test_mixed_literal_heavy_routing(dev, monkeypatch, codec):
    """decompress() sends streams stored at >= LANES_RATIO of their size to
    the lane decoder and the rest to the library's choice, two launches:
    interleaved incompressible and text streams come back in order with
    their own statuses (a short capacity on one of each kind)."""
    monkeypatch.delenv("STROM_DECOMP_PAR", raising=False)
    from nvme_strom_amd.ops import decompress as D
    rng = np.random.default_rng(11)
    words = [b"select", b"from", b"where", b"gpu", b"hbm"]
    pays = []
    for i in range(24):
        if i % 3 == 0:
            pays.append(rng.integers(0, 256, 20000 + 97 * i, dtype=np.uint8).tobytes())
        else:
            pays.append(b" ".join(words[j] for j in rng.integers(0, 5, 9000 + 13 * i)))
    enc = D.lz4_compress if codec == "lz4" else D.snappy_compress
    comp = [enc(p) for p in pays]
    assert any(len(c) >= D.LANES_RATIO * len(p) for c, p in zip(comp, pays))
    assert any(len(c) < D.LANES_RATIO * len(p) for c, p in zip(comp, pays))
    sizes = [len(p) for p in pays]
    sizes[3] -= 1                       # literal-heavy, one byte short
    sizes[4] -= 1                       # compressible, one byte short
    cid = D.LZ4 if codec == "lz4" else D.SNAPPY
    st, outs = _run(cid, comp, sizes, dev)
    for i, p in enumerate(pays):
        if i in (3, 4):
            assert st[i] < 0, (i, st[i])
        else:
            assert st[i] == len(p) and outs[i] == p, (i, st[i])


@pytest.mark.parametrize("which", ["ours", "pyarrow"])
def test_lz4_raw(dev, which):
    from nvme_strom_amd.ops import decompress as D
    pays = _payloads()
    if which == "pyarrow":
        pa = pytest.importorskip("pyarrow")
        comp = [pa.compress(p, codec="lz4_raw", asbytes=True) if p else D.lz4_compress(p) for p in pays]
    else:
        comp = [D.lz4_compress(p) for p in pays]
    st, outs = _run(D.LZ4, comp, [len(p) for p in pays], dev)
    assert list(st) == [len(p) for p in pays]
    assert outs == pays


@pytest.mark.parametrize("g", [1, 2, 3, 4, 6, 8, 16, 32, "par256", "par512", "par8192"])
@pytest.mark.parametrize("codec", ["lz4", "snappy"])
def test_decoder_geometries(dev, monkeypatch, g, codec):
    """Every streams-per-wave variant of the lane-group decoder
    (STROM_DECOMP_G, the block-parallel decoder switched off) decodes the
    same payloads: the fast LZ4 step's pass width differs per geometry (a
    length-15 match nibble must still take the extended-length path);
    3 / 2 / 6 = the large-ring few-stream geometries; "par256" / "par512" /
    "par8192" = the block-parallel decoder's three builds (lz4par.hip,
    lz4par_nt512.hip, lz4par_nt512_ob8k.hip)."""
    pa = pytest.importorskip("pyarrow")
    from nvme_strom_amd.ops import decompress as D
    if str(g).startswith("par"):
        monkeypatch.setenv("STROM_DECOMP_PAR", g[3:])
    else:
        monkeypatch.setenv("STROM_DECOMP_PAR", "0")
        monkeypatch.setenv("STROM_DECOMP_G", str(g))
    pays = _payloads()
    name, cid = ("lz4_raw", D.LZ4) if codec == "lz4" else ("snappy", D.SNAPPY)
    comp = [pa.compress(p, codec=name, asbytes=True) if p else
            (D.lz4_compress(p) if codec == "lz4" else D.snappy_compress(p)) for p in pays]
    st, outs = _run(cid, comp, [len(p) for p in pays], dev)
    assert list(st) == [len(p) for p in pays]
    assert outs == pays


@pytest.mark.parametrize("which", ["ours", "pyarrow"])
def test_snappy(dev, which):
    from nvme_strom_amd.ops import decompress as D
    pays = _payloads()
    if which == "pyarrow":
        pa = pytest.importorskip("pyarrow")
        comp = [pa.compress(p, codec="snappy", asbytes=True) for p in pays]
    else:
        comp = [D.snappy_compress(p) for p in pays]
    st, outs = _run(D.SNAPPY, comp, [len(p) for p in pays], dev)
    assert list(st) == [len(p) for p in pays]
    assert outs == pays


@pytest.mark.parametrize("g", ["auto", "lanes", "256", "512", "8192"])
def test_lz4_frame_linked_blocks_from_pyarrow(dev, monkeypatch, g):
    """pyarrow's 'lz4' codec = LZ4 frame with linked 64 KiB blocks: matches
    may reach into the previous block (lane groups: the LDS history ring;
    block-parallel: stored output read back)."""
    pa = pytest.importorskip("pyarrow")
    if g != "auto":
        monkeypatch.setenv("STROM_DECOMP_PAR", "0" if g == "lanes" else g)
    from nvme_strom_amd.ops import decompress as D
    pays = [p for p in _payloads() if p]
    frames = [pa.compress(p, codec="lz4", asbytes=True) for p in pays]
    infos = [D.parse_lz4_frame_header(f) for f in frames]
    streams = [f[i.data_offset:] for f, i in zip(frames, infos)]
    codec = D.LZ4_FRAME_BCS if infos[0].block_checksum else D.LZ4_FRAME
    st, outs = _run(codec, streams, [len(p) for p in pays], dev)
    assert list(st) == [len(p) for p in pays]
    assert outs == pays


@pytest.mark.parametrize("g", ["0", "256", "512", "8192"])
def test_malformed_streams_report_errors(dev, monkeypatch, g):
    from nvme_strom_amd.ops import decompress as D
    monkeypatch.setenv("STROM_DECOMP_PAR", g)
    rng = np.random.default_rng(5)
    junk = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (10, 1000, 5000)]
    good = D.lz4_compress(b"hello world " * 1000)
    st, _ = _run(D.LZ4, junk + [good, good[:-3]], [4096, 4096, 4096, 12000, 12000], dev)
    assert st[3] == 12000
    assert (st[:3] < 0).all() or (st[:3] <= 4096).all()   # bounded, never out of range
    st, _ = _run(D.SNAPPY, junk, [4096] * 3, dev)
    assert (st < 0).all()


# ---------------------------------------------------------------------- zstd
@pytest.fixture(params=[0, 1, 2], ids=["wave", "fp", "lp"])
def zmode(request, dev):
    """Every zstd decoder: one wave per stream, frame-parallel (the blocks of
    a frame on the waves of a workgroup) and lane-parallel (the Arrow scan's
    default: walk, entropy groups, executions; checked against its host
    twin's LP-taken count as well)."""
    from nvme_strom_amd import _native as N
    from nvme_strom_amd.ops import decompress as D
    if request.param == 2:
        _ZSTD_ROUTE["mode"] = D.ZSTD_LP
    else:
        N.lib().strom_zstd_fp_mode(request.param)
    yield request.param
    _ZSTD_ROUTE["mode"] = None
    N.lib().strom_zstd_fp_mode(-1)


@pytest.mark.parametrize("level", [-5, 1, 3, 19])
def test_zstd_from_pyarrow(dev, zmode, level):
    """zstd.hip (one wavefront per stream, or frame-parallel) == the input,
    for pyarrow's zstd frames of every payload kind in one launch."""
    pa = pytest.importorskip("pyarrow")
    from nvme_strom_amd.ops import decompress as D
    codec = pa.Codec("zstd", compression_level=level)
    pays = _payloads()
    comp = [codec.compress(p, asbytes=True) for p in pays]
    st, outs = _run(D.ZSTD, comp, [len(p) for p in pays], dev)
    assert list(st) == [len(p) for p in pays]
    assert outs == pays


def test_zstd_randomized_differential(dev, zmode):
    """200 random payloads (mixtures of text, runs, random bytes, ints and
    floats, 0 B - 400 KB) at random levels -7..19 in one launch: every
    block / literal / table mode pyarrow's encoder picks, raw blocks inside
    compressed frames, decoded on the GPU == the input."""
    pa = pytest.importorskip("pyarrow")
    from nvme_strom_amd.ops import decompress as D
    rng = np.random.default_rng(2024)
    words = [b"alpha", b"beta", b"gamma", b"nvme", b"strom", b"hbm", b"gfx950"]
    pays, comp = [], []
    for i in range(200):
        parts = []
        for _ in range(int(rng.integers(1, 6))):
            k = int(rng.integers(0, 5))
            n = int(rng.integers(0, 120_000))
            if k == 0:
                parts.append(b" ".join(words[j] for j in rng.integers(0, len(words), n // 5 + 1))[:n])
            elif k == 1:
                parts.append(bytes([int(rng.integers(0, 256))]) * n)
            elif k == 2:
                parts.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
            elif k == 3:
                parts.append(rng.integers(0, int(rng.integers(2, 1 << 40)), n // 8 + 1,
                                          dtype=np.int64).tobytes())
            else:
                parts.append(rng.random(n // 8 + 1).tobytes())
        p = b"".join(parts)[: int(rng.integers(0, 400_000))]
        level = int(rng.integers(-7, 20))
        pays.append(p)
        comp.append(pa.Codec("zstd", compression_level=level).compress(p, asbytes=True))
    st, outs = _run(D.ZSTD, comp, [len(p) for p in pays], dev)
    assert list(st) == [len(p) for p in pays]
    assert outs == pays


@pytest.mark.parametrize("lp", [False, True], ids=["slots", "lp"])
def test_zstd_scratch_cache_many_streams(dev, lp):
    """Decodes on 12 HIP streams in turn: the library's per-stream literal
    scratch (or LP entry pool) is capped (least recently used evicted) and
    every decode stays right; strom_zstd_release() frees what is left."""
    pa = pytest.importorskip("pyarrow")
    from nvme_strom_amd import _native as N
    from nvme_strom_amd.ops import decompress as D
    rng = np.random.default_rng(31)
    pays = [rng.integers(0, 1000, 30000, dtype=np.int64).tobytes() for _ in range(6)]
    comp = [pa.Codec("zstd").compress(p, asbytes=True) for p in pays]
    src = b"".join(comp)
    offs = np.cumsum([0] + [len(c) for c in comp])[:-1]
    doffs = np.arange(len(pays)) * len(pays[0])
    descs = D.make_descs([(int(o), len(c), int(do), len(p))
                          for o, c, do, p in zip(offs, comp, doffs, pays)])
    d_src = _t(src + b"\0", dev)
    d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
    want = b"".join(pays)
    for k in range(12):
        st = torch.cuda.Stream(device=dev)
        dst = torch.zeros(len(want), dtype=torch.uint8, device=dev)
        status = torch.empty(len(pays), dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        D.decompress_async(D.ZSTD, d_src, dst, d_desc, status, stream=st,
                           zstd_mode=D.ZSTD_LP if lp else None)
        st.synchronize()
        assert status.cpu().tolist() == [len(p) for p in pays], k
        assert dst.cpu().numpy().tobytes() == want, k
    assert N.lib().strom_zstd_release() == 0


def test_zstd_mutants_bounded(dev, zmode):
    """Byte-flipped and truncated frames in one launch with good ones: every
    status is an error or within the stream's capacity and the good streams
    (placed before the mutants' outputs) decode exactly (LP: statuses equal
    the host twin's, and the LP-taken count too — _run_lp)."""
    pa = pytest.importorskip("pyarrow")
    from nvme_strom_amd.ops import decompress as D
    rng = np.random.default_rng(99)
    pays = [p for p in _payloads() if len(p) > 100]
    frames = [pa.Codec("zstd", compression_level=int(rng.integers(1, 10))).compress(p, asbytes=True)
              for p in pays]
    streams, sizes = list(frames), [len(p) for p in pays]
    for k in range(40):
        f = bytearray(frames[k % len(frames)])
        if k % 5 == 4:
            f = f[:int(rng.integers(1, len(f)))]
        else:
            for _ in range(int(rng.integers(1, 4))):
                j = int(rng.integers(0, len(f)))
                f[j] ^= 1 << int(rng.integers(0, 8))
        streams.append(bytes(f))
        sizes.append(len(pays[k % len(frames)]))
    st, outs = _run(D.ZSTD, streams, sizes, dev)
    good = len(frames)
    assert list(st[:good]) == sizes[:good] and outs[:good] == pays
    assert all(x < 0 or x <= n for x, n in zip(st[good:].tolist(), sizes[good:]))


def test_zstd_content_checksum(dev, zmode):
    """Frames with the content-checksum flag verify on the GPU (XXH64 on
    lanes 0..3 over each frame's output); a flipped checksum bit gives -5."""
    pa = pytest.importorskip("pyarrow")
    xxhash = pytest.importorskip("xxhash")
    import struct
    from nvme_strom_amd.ops import decompress as D
    pays = [p for p in _payloads() if p]
    comp = []
    for p in pays:
        f = bytearray(pa.Codec("zstd").compress(p, asbytes=True))
        f[4] |= 0x04
        comp.append(bytes(f) + struct.pack("<I", xxhash.xxh64_intdigest(p, 0) & 0xFFFFFFFF))
    bad = comp[0][:-1] + bytes([comp[0][-1] ^ 0x80])
    st, outs = _run(D.ZSTD, comp + [bad], [len(p) for p in pays] + [len(pays[0])], dev)
    assert list(st[:-1]) == [len(p) for p in pays]
    assert outs[:-1] == pays
    assert st[-1] == -5


def test_zstd_persistent_slots_and_arrow(dev, zmode):
    """More streams than scratch slots (each workgroup loops over streams
    and reuses its literal slot), Arrow IPC buffers incl. a stored one, and
    malformed streams reported without touching memory out of range."""
    pa = pytest.importorskip("pyarrow")
    from nvme_strom_amd import _native as N
    from nvme_strom_amd.ops import decompress as D
    rng = np.random.default_rng(21)
    pays = [rng.integers(0, 1_000_000, int(n), dtype=np.int64).tobytes()
            for n in rng.integers(1000, 70000, 40)]
    bufs = [D.arrow_zstd_buffer(p, pa.Codec("zstd").compress(p, asbytes=True)) for p in pays]
    bufs[3] = b"\xff" * 8 + pays[3]
    good = len(bufs)
    junk = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (10, 1000, 5000)]
    trunc = bufs[0][: len(bufs[0]) // 2]
    streams = bufs + junk + [trunc]
    sizes = [len(p) for p in pays] + [4096] * 3 + [len(pays[0])]
    src = b"".join(streams)
    offs = np.cumsum([0] + [len(x) for x in streams])[:-1]
    doffs = np.cumsum([0] + sizes)[:-1]
    descs = D.make_descs([(int(o), len(x), int(do), n) for o, x, do, n in zip(offs, streams, doffs, sizes)])
    d_src = _t(src + b"\0", dev)
    dst = torch.zeros(sum(sizes) + 64, dtype=torch.uint8, device=dev)
    guard = dst[sum(sizes):]
    d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
    status = torch.empty(len(streams), dtype=torch.int32, device=dev)
    if zmode == 2:
        # the LP pool is the library's; the capacity past the outputs (the
        # guard) is part of dst, so it sizes the pool but is never written
        D.decompress_async(D.ARROW_ZSTD, d_src, dst, d_desc, status, zstd_mode=D.ZSTD_LP)
    else:
        sz = np.zeros(2, np.uint64)
        N.lib().strom_zstd_scratch_sizes(sz.ctypes.data)
        scratch = torch.empty(3 * int(sz[zmode]), dtype=torch.uint8, device=dev)   # 3 slots
        rc = N.lib().strom_decompress_zstd(D.ARROW_ZSTD, d_src.data_ptr(), dst.data_ptr(),
                                            d_desc.data_ptr(), len(streams), status.data_ptr(),
                                            scratch.data_ptr(), scratch.numel(), None)
        assert rc == 0
    st = status.cpu().numpy()
    out = dst.cpu().numpy().tobytes()
    assert list(st[:good]) == sizes[:good]
    for p, do in zip(pays, doffs[:good]):
        assert out[int(do):int(do) + len(p)] == p
    assert (st[good:] < 0).all() or (st[good:] <= np.array(sizes[good:])).all()
    assert st[-1] < 0
    assert int(guard.count_nonzero()) == 0


# -------------------------------------------------------------- column filter
@pytest.mark.parametrize("dtype", [torch.int32, torch.int64, torch.float32, torch.float64])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 255 * 64 + 7, 1_000_003])
def test_column_filter(dev, dtype, n):
    from nvme_strom_amd.ops.colfilter import bitmap_to_indices, column_filter
    rng = np.random.default_rng(2)
    v = rng.integers(-1000, 1000, n)
    vt = torch.from_numpy(v).to(dtype).to(dev)
    valid_bits = rng.random(n) > 0.1
    valid = np.packbits(valid_bits, bitorder="little")
    vb = torch.from_numpy(np.concatenate([valid, np.zeros(64, np.uint8)])).to(dev)
    bm, cnt = column_filter(vt, -100, 250, vb)
    ref = (v >= -100) & (v <= 250) & valid_bits
    assert cnt == int(ref.sum())
    got = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(got, ref)
    idx = bitmap_to_indices(bm, n, cnt)
    assert np.array_equal(idx.cpu().numpy(), np.nonzero(ref)[0].astype(np.int32))


@pytest.mark.parametrize("density", [0.0, 0.003, 0.5, 1.0])
def test_bitmap_to_indices_many_tiles(dev, density):
    """Single-pass look-back compaction over ~1200 tiles vs numpy.nonzero."""
    from nvme_strom_amd.ops.colfilter import bitmap_to_indices
    n = 20_000_037
    bits = np.random.default_rng(7).random(n) < density
    packed = np.packbits(bits, bitorder="little")
    packed = np.concatenate([packed, np.full((-len(packed)) % 8 + 8, 0xFF, np.uint8)])  # junk past n
    bm = torch.from_numpy(packed.view(np.uint64).copy()).to(dev)
    ref = np.nonzero(bits)[0]
    idx = bitmap_to_indices(bm, n, int(bits.sum()))
    assert np.array_equal(idx.cpu().numpy().astype(np.int64), ref)
