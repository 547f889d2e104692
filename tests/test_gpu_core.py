"""GPU tests (MI355X): kernel numerics vs host references, SSD→HBM end to end."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nvme_strom_amd as S
    S.configure(gpu_emulation=0, backend="uring", max_request=1 << 20, workers=4,
                pgcache_probe=1, direct_io=1)
    return S


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n,chunk", [(1, 16), (3, 16), (4, 16), (17, 16), (1000, 1024),
                                     (8192 * 5 + 77, 8192), (1 << 20, 1 << 20),
                                     ((3 << 20) + 4096 + 5, 1 << 16), (100000, 4096),
                                     # workgroup-per-chunk schedule: parts of 1-KiB rows,
                                     # a 2-byte last part, a 3-byte tail chunk
                                     ((5 << 20) + 16386, 1 << 20), ((1 << 20) + 3, 1 << 20),
                                     (3 * 20000 + 7, 20000)])
def test_crc32c_chunks_vs_host(S, n, chunk):
    from nvme_strom_amd.ops import verify as V
    data = np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8)
    dev = V.u32(V.crc32c_chunks(_dev(data), chunk))
    ref = [S.crc32c_host(data[i:i + chunk].tobytes()) for i in range(0, n, chunk)]
    assert list(dev) == ref
    assert V.crc32c(_dev(data), chunk=chunk) == S.crc32c_host(data.tobytes())


def test_crc32c_known_vector(S):
    from nvme_strom_amd.ops import verify as V
    assert S.crc32c_host(b"123456789") == 0xE3069283
    t = _dev(np.frombuffer(b"123456789" + b"\0" * 7, dtype=np.uint8))
    assert V.crc32c(t, nbytes=9, chunk=16) == 0xE3069283


def test_scatter_gather(S):
    from nvme_strom_amd.ops.reorder import chunk_gather, chunk_scatter
    ch, n = 8192, 97
    src = torch.randint(0, 256, (n * ch,), dtype=torch.uint8, device="cuda")
    perm = np.random.default_rng(0).permutation(n).astype(np.uint32)
    dst = torch.empty_like(src)
    chunk_scatter(src, dst, perm, ch)
    ref = torch.empty_like(src).view(n, ch)
    ref[torch.from_numpy(perm.astype(np.int64)).cuda()] = src.view(n, ch)
    assert torch.equal(dst.view(n, ch), ref)
    back = torch.empty_like(src)
    chunk_gather(dst, back, perm, ch)
    assert torch.equal(back, src)


def test_verify_and_fill(S):
    from nvme_strom_amd.ops import verify as V
    t = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    V.fill_pattern(t, 0x41424344)
    assert V.verify_pattern(t, 0x41424344) == (0, -1)
    t[4096 + 5] = 0
    t[8000] = 1
    assert V.verify_pattern(t, 0x41424344) == (2, 4096 + 4)
    u = t.clone()
    assert V.verify_equal(t, u) == (0, -1)
    u[12] = 7
    assert V.verify_equal(t, u)[1] == 12


def _mkfile(tmp_path, n, seed=0):
    data = np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)
    p = str(tmp_path / f"f{seed}.bin")
    with open(p, "wb") as f:
        f.write(data.tobytes())
        f.flush()
        os.fsync(f.fileno())
    fd = os.open(p, os.O_RDONLY)
    os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    os.close(fd)
    return p, data


@pytest.mark.parametrize("backend", ["uring", "psync"])
def test_load_file_end_to_end(S, tmp_path, backend):
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.tensor import load_file
    S.configure(backend=backend)
    p, data = _mkfile(tmp_path, (16 << 20) + 12345)
    t = load_file(p, device="cuda", chunk_sz=1 << 16, window=4 << 20)
    assert torch.equal(t.cpu(), torch.from_numpy(data))
    assert V.crc32c(t) == S.crc32c_host(data.tobytes())
    S.configure(backend="uring")


@pytest.mark.parametrize("coalesce", [0, 1])
def test_worker_copy_coalescing(S, tmp_path, coalesce):
    """128 KiB requests through the SDMA path (ingest grid off, past the
    64 KiB BAR cut) land byte-exact whether adjacent staged copies are merged
    or not."""
    from nvme_strom_amd.tensor import load_file
    S.configure(max_request=128 << 10, coalesce=coalesce, ingest=0)
    try:
        p, data = _mkfile(tmp_path, (24 << 20) + 8192, seed=9)
        t = load_file(p, device="cuda", chunk_sz=1 << 16, window=8 << 20)
        assert torch.equal(t.cpu(), torch.from_numpy(data))
    finally:
        S.configure(max_request=1 << 20, coalesce=1, ingest=1)


@pytest.mark.parametrize("req", [4096, 16384, 65536, 262144, 1 << 20, 4 << 20])
def test_ingest_grid_request_sizes(S, tmp_path, req):
    """The GPU ingest grid pulls staged reads into HBM byte-exact at every
    request size (pieces of ingest_piece bytes).  Two files with different
    bytes go through the same pinned staging slots one after the other, so a
    stale GPU-cached copy of a refilled slot would show as a mismatch."""
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.tensor import load_file
    S.configure(max_request=req, ingest=1, workers=4)
    before = S.ingest_info(0)
    assert before and before["available"]
    try:
        for seed in (21, 22):
            p, data = _mkfile(tmp_path, (12 << 20) + 4096, seed=seed)
            t = load_file(p, device="cuda", chunk_sz=min(req, 1 << 16), window=4 << 20)
            assert torch.equal(t.cpu(), torch.from_numpy(data)), seed
            assert V.crc32c(t) == S.crc32c_host(data.tobytes())
        after = S.ingest_info(0)
        assert after["posted"] >= before["posted"] + (24 << 20) // max(req, 256 << 10) // 2
        assert after["outstanding"] == 0
    finally:
        S.configure(max_request=1 << 20, ingest=1)


def test_ingest_grid_stops_when_idle(S, tmp_path):
    """A device-wide synchronize returns once the engine is idle: the ingest
    grid is a persistent kernel, so the workers stop it before sleeping."""
    import time
    from nvme_strom_amd.tensor import load_file
    S.configure(ingest=1)
    p, data = _mkfile(tmp_path, 8 << 20, seed=23)
    t = load_file(p, device="cuda", chunk_sz=1 << 16, window=2 << 20)
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 5.0
    assert torch.equal(t.cpu(), torch.from_numpy(data))


def test_pread_gpu_visible_to_next_kernel(S, tmp_path):
    """Posted HDP flush (hdp_sync=0): bytes stored through the BAR by
    pread_gpu are seen by a kernel launched right after it returns — 1000
    distinct 4 KiB offsets, each checked by its own CRC kernel."""
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.tensor import HbmBuffer
    S.configure(hdp_sync=0, bar_map=1)
    n = 1000
    p, data = _mkfile(tmp_path, 16 << 20, seed=31)
    fd = os.open(p, os.O_RDONLY)
    offs = np.random.default_rng(3).choice((16 << 20) // 4096, n, replace=False) * 4096
    crcs = []
    with HbmBuffer(n * 4096, "cuda") as hb:
        for i, off in enumerate(offs.tolist()):
            assert S.pread_gpu(hb.handle, i * 4096, fd, off, 4096) == 4096
            crcs.append(V.crc32c_chunks(hb.tensor[i * 4096:(i + 1) * 4096], 4096))
        got = [int(V.u32(c)[0]) for c in crcs]
    os.close(fd)
    ref = [S.crc32c_host(data[o:o + 4096].tobytes()) for o in offs.tolist()]
    bad = [i for i in range(n) if got[i] != ref[i]]
    assert not bad, f"{len(bad)} stale reads, first at {bad[:5]}"


def test_pread_gpu_visible_to_sdma_readback(S, tmp_path):
    """the posted HDP flush is also enough for a copy-engine
    consumer — each 4 KiB pread_gpu is read back with a D2H copy started
    right after it returns (no kernel launch in between), 500 offsets."""
    from nvme_strom_amd.tensor import HbmBuffer
    S.configure(hdp_sync=0, bar_map=1)
    n = 500
    p, data = _mkfile(tmp_path, 8 << 20, seed=37)
    fd = os.open(p, os.O_RDONLY)
    offs = np.random.default_rng(4).choice((8 << 20) // 4096, n, replace=False) * 4096
    host = torch.empty(4096, dtype=torch.uint8, pin_memory=True)
    bad = []
    with HbmBuffer(n * 4096, "cuda") as hb:
        for i, off in enumerate(offs.tolist()):
            assert S.pread_gpu(hb.handle, i * 4096, fd, off, 4096) == 4096
            host.copy_(hb.tensor[i * 4096:(i + 1) * 4096])      # hipMemcpy D2H
            if not np.array_equal(host.numpy(), data[off:off + 4096]):
                bad.append(i)
    os.close(fd)
    assert not bad, f"{len(bad)} stale D2H reads, first at {bad[:5]}"


def test_pread_gpu_visible_to_other_stream_kernel(S, tmp_path):
    """a peer-style consumer — a kernel on ANOTHER stream
    (created beforehand, as RCCL's would be), launched without any host sync
    after each 4 KiB pread_gpu returns — sees the bytes, with the posted HDP
    flush of the synchronous path (hdp_sync=2 default) and with hdp_sync=0."""
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.tensor import HbmBuffer
    n = 500
    p, data = _mkfile(tmp_path, 8 << 20, seed=41)
    fd = os.open(p, os.O_RDONLY)
    offs = np.random.default_rng(5).choice((8 << 20) // 4096, n, replace=False) * 4096
    side = torch.cuda.Stream()
    ref = [S.crc32c_host(data[o:o + 4096].tobytes()) for o in offs.tolist()]
    for mode in (2, 0):
        S.configure(hdp_sync=mode, bar_map=1)
        crcs = []
        with HbmBuffer(n * 4096, "cuda") as hb:
            for i, off in enumerate(offs.tolist()):
                assert S.pread_gpu(hb.handle, i * 4096, fd, off, 4096) == 4096
                with torch.cuda.stream(side):
                    crcs.append(V.crc32c_chunks(hb.tensor[i * 4096:(i + 1) * 4096], 4096))
            side.synchronize()
            got = [int(V.u32(c)[0]) for c in crcs]
        bad = [i for i in range(n) if got[i] != ref[i]]
        assert not bad, f"hdp_sync={mode}: {len(bad)} stale reads, first at {bad[:5]}"
    os.close(fd)
    S.configure(hdp_sync=2)


def test_read_chunks_hybrid_reorder(S, tmp_path):
    """Page-cache chunks land at the tail via the write-back buffer; the
    reader scatters everything back into the requested order on the GPU."""
    from nvme_strom_amd.tensor import FileReader, HbmBuffer
    ch, n = 8192, 256
    p, data = _mkfile(tmp_path, ch * n, seed=3)
    fd = os.open(p, os.O_RDONLY)
    os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_RANDOM)
    for c in (5, 6, 100, 200, 255):
        os.pread(fd, ch, c * ch)
    os.close(fd)
    req = np.random.default_rng(1).permutation(n).astype(np.uint32)
    with FileReader(p, chunk_sz=ch, max_chunks=n) as rd, HbmBuffer(n * ch, "cuda") as hb:
        res, landed = rd.submit(hb, 0, req)
        rd.finish(res)
        assert res.nr_ram >= 1
        rd2 = FileReader(p, chunk_sz=ch, max_chunks=n)
        out = rd2.read_chunks(hb, 0, req)
        rd2.close()
        ref = data.reshape(n, ch)[req.astype(np.int64)].reshape(-1)
        assert torch.equal(out.cpu(), torch.from_numpy(ref))


def test_stream_loader_verify(S, tmp_path):
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    p, data = _mkfile(tmp_path, 64 << 20, seed=5)
    ld = StreamLoader(p, segment_sz=8 << 20, nr_segments=4, chunk_sz=8192, device="cuda", depth=3)
    st = ld.run(0, 64 << 20, verify=True)
    assert st.crc_mismatch == 0
    assert st.nr_ssd + st.nr_ram == (64 << 20) // 8192
    ld.close()


def test_map_real_hbm_and_info(S):
    t = torch.empty(3 << 20, dtype=torch.uint8, device="cuda")
    m = S.map_gpu_memory(t.data_ptr(), t.numel())
    info = S.info_gpu_memory(m.handle)
    assert info["map_length"] == info["map_offset"] + t.numel()
    m.unmap()
    # host memory is not GPU memory when emulation is off
    h = np.zeros(1 << 16, dtype=np.uint8)
    with pytest.raises(S.StromError):
        S.map_gpu_memory(h.ctypes.data, h.nbytes)


def test_pread_gpu_mixed_cache(S, tmp_path):
    """pread_gpu keeps file order even when some pages come from the page
    cache (landed at the tail, written through the BAR when available)."""
    from nvme_strom_amd.tensor import HbmBuffer
    p, data = _mkfile(tmp_path, 4 << 20, seed=11)
    fd = os.open(p, os.O_RDONLY)
    os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_RANDOM)
    for pg in (1, 2, 7, 60, 61):
        os.pread(fd, 4096, (256 + pg) * 4096)
    with HbmBuffer(2 << 20, "cuda") as hb:
        for bar in (1, 0):
            S.configure(bar_map=bar)
            hb2 = HbmBuffer(2 << 20, "cuda")
            n = S.pread_gpu(hb2.handle, 4096, fd, 256 * 4096, 128 * 4096)
            assert n == 128 * 4096
            got = hb2.tensor[4096:4096 + n].cpu().numpy()
            assert np.array_equal(got, data[256 * 4096:256 * 4096 + n])
            hb2.close()
    S.configure(bar_map=1)
    os.close(fd)


def test_latency_4k(S, tmp_path):
    import time
    from nvme_strom_amd.tensor import FileReader, HbmBuffer
    p, data = _mkfile(tmp_path, 64 << 20, seed=9)
    with FileReader(p, chunk_sz=4096, max_chunks=1) as rd, HbmBuffer(1 << 20, "cuda") as hb:
        lat = []
        for cid in np.random.default_rng(0).integers(0, (64 << 20) // 4096, 300):
            t0 = time.perf_counter()
            res, _ = rd.submit(hb, 0, np.array([cid], dtype=np.uint32))
            rd.finish(res)
            lat.append(time.perf_counter() - t0)
            got = hb.tensor[:4096].cpu().numpy()
            assert np.array_equal(got, data[cid * 4096:(cid + 1) * 4096])
        assert np.median(lat) < 0.01


def test_export_dmabuf_offsets(S):
    """MAP_GPU_MEMORY under the kernel provider registers the dma-buf of the
    whole allocation plus the range's offset in it (tensors are usually
    sub-allocations of a caching-allocator block)."""
    import ctypes as C
    from nvme_strom_amd import _native as N
    t = torch.empty(8 << 20, dtype=torch.uint8, device="cuda")
    lib = N.lib()
    fds, offs = [], []
    try:
        for delta in (0, (1 << 20) + 4096):
            fd, off = C.c_int(-1), C.c_uint64(0)
            assert lib.strom_export_dmabuf(t.data_ptr() + delta, 4096, C.byref(fd), C.byref(off)) == 0
            assert fd.value >= 0
            fds.append(fd.value)
            offs.append(off.value)
        assert offs[1] - offs[0] == (1 << 20) + 4096
        # a dma-buf reports its size through lseek(SEEK_END)
        assert os.lseek(fds[0], 0, os.SEEK_END) >= offs[0] + (8 << 20)
        h = np.zeros(4096, dtype=np.uint8)
        assert lib.strom_export_dmabuf(h.ctypes.data, 4096, C.byref(C.c_int()), C.byref(C.c_uint64())) < 0
    finally:
        for fd in fds:
            os.close(fd)


def test_freed_allocation_detaches_mapping(S, tmp_path):
    """hipFree of a mapped range (torch: del + empty_cache) is caught at the
    next SSD2GPU: -ENOENT, handle gone (reference free callback,
    kmod/pmemmap.c:150-208) — nothing is written into recycled memory."""
    import errno
    path = str(tmp_path / "f.bin")
    with open(path, "wb") as f:
        f.write(os.urandom(1 << 20))
    fd = os.open(path, os.O_RDONLY)
    S.evict_file(fd)
    try:
        t = torch.empty(8 << 20, dtype=torch.uint8, device="cuda")
        m = S.map_gpu_memory(t.data_ptr(), t.numel())
        # the large-BAR alias is set up (probe on a private allocation)
        assert S.session().lib.strom_gpu_bar_bytes(m.handle) >= t.numel()
        r = S.memcpy_ssd2gpu(m.handle, 0, fd, np.arange(4, dtype=np.uint32), 65536)
        S.memcpy_wait(r.dma_task_id)
        before = S.gpu_detached()
        del t
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        with pytest.raises(S.StromError) as e:
            S.memcpy_ssd2gpu(m.handle, 0, fd, np.arange(4, dtype=np.uint32), 65536)
        assert e.value.errno == errno.ENOENT
        assert S.gpu_detached() == before + 1
        assert m.handle not in S.list_gpu_memory()
        m.handle = 0
    finally:
        os.close(fd)


def test_stripe_set_to_hbm(S, tmp_path):
    """A stripe set over 3 member files loads into HBM in logical order
    (requests split per member, run concurrently); CRC on the GPU."""
    from nvme_strom_amd.ops import verify as V
    from nvme_strom_amd.tensor import load_file
    unit = 256 << 10
    data = np.random.default_rng(12).integers(0, 256, (24 << 20) + 12345, dtype=np.uint8)
    paths = [str(tmp_path / f"m{k}.bin") for k in range(3)]
    size = S.write_striped(paths, data, unit)
    for p in paths:
        fd = os.open(p, os.O_RDONLY)
        S.evict_file(fd)
        os.close(fd)
    with S.StripeSet(paths, unit) as ss:
        t = load_file(ss, "cuda", chunk_sz=1 << 20)
        torch.cuda.synchronize()
        assert t.numel() == size
        assert V.crc32c(t) == S.crc32c_host(data.tobytes())


def test_default_stream_runs_while_grid_reads(S, tmp_path):
    """Work on PyTorch's default stream, and a side stream ordered after it
    by an event (as the Arrow scan's decode streams are), goes through while
    a large read is still landing through the persistent ingest grid — the
    grid never holds other streams' work until it goes idle."""
    import time
    from nvme_strom_amd.tensor import FileReader, HbmBuffer
    S.configure(ingest=1)
    n = 1 << 30
    p = str(tmp_path / "big.bin")
    with open(p, "wb") as f:
        blk = np.random.default_rng(31).integers(0, 256, size=64 << 20, dtype=np.uint8).tobytes()
        for _ in range(n // len(blk)):
            f.write(blk)
    hb = HbmBuffer(n, "cuda")
    chunk = 1 << 20
    r = FileReader(p, chunk_sz=chunk, max_chunks=n // chunk)
    try:
        S.evict_file(r.fd)
        x = torch.ones(1 << 20, device="cuda")
        side = torch.cuda.Stream()
        y = x * 2                               # kernel code loaded before timing
        with torch.cuda.stream(side):
            z = x * 3
        torch.cuda.synchronize()
        res, _ = r.submit(hb, 0, np.arange(n // chunk, dtype=np.uint32))
        time.sleep(0.002)                       # the grid is resident now
        t0 = time.perf_counter()
        y = x * 2                               # default stream
        # a side stream ordered after the default stream (an event recorded
        # on it), as the Arrow scan's decode streams were
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            z = x * 3
        side.synchronize()
        torch.cuda.current_stream().synchronize()
        t1 = time.perf_counter()
        r.finish(res)
        t2 = time.perf_counter()
        assert float(y[0]) == 2.0 and float(z[0]) == 3.0
        # the rest of a 1 GiB read takes tens of ms; the default stream
        # came back long before it landed
        assert t2 - t0 > 0.01, (t1 - t0, t2 - t0)
        assert (t1 - t0) < 0.3 * (t2 - t0), (t1 - t0, t2 - t0)
    finally:
        r.close()
        hb.close()
