"""End-to-end engine semantics on the CPU (real files, io_uring/pread
backends, host memory standing in for HBM via gpu_emulation).

Covers the reference semantics of do_memcpy_ssd2gpu / do_memcpy_ssd2ram
(kmod/nvme_strom.c:1488-1604, 1767-1884): relseg modulo addressing, the
page-cache majority score, SSD-head / RAM-tail landing order with chunk_ids
rewritten, request merging, EOF handling, and error propagation via WAIT.
"""
import errno
import os

import numpy as np
import pytest

CH = 8192


def _open(path):
    return os.open(path, os.O_RDONLY)


def _host_target(nbytes):
    buf = np.zeros(nbytes + 65536, dtype=np.uint8)
    base = buf.ctypes.data
    off = (-base) % 65536          # 64 KiB aligned view, like a GPU page
    return buf, buf[off:off + nbytes]


def _chunks(data, ids, chunk=CH, relseg=0):
    out = []
    for cid in ids:
        c = (cid % relseg) if relseg else cid
        out.append(data[c * chunk:(c + 1) * chunk])
    return np.concatenate(out)


@pytest.mark.parametrize("backend", ["uring", "psync", "cache"])
def test_ssd2ram_identity_and_permutation(strom, rand_file, backend):
    # cache: worker reads through the buffered descriptor (the engine-ceiling
    # mode of tools/ceiling_bench.py), the page-cache probe off
    strom.configure(backend=backend, pgcache_probe=int(backend != "cache"))
    assert strom.config_get("backend") == backend
    path, data = rand_file(64 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(64 * CH) as buf:
            ids = np.arange(64, dtype=np.uint32)
            r = strom.memcpy_ssd2ram(buf.address, fd, ids, CH)
            strom.memcpy_wait(r.dma_task_id)
            assert r.nr_ssd + r.nr_ram == 64
            assert np.array_equal(buf.array[:64 * CH], data)
            perm = np.random.default_rng(1).permutation(64).astype(np.uint32)
            r = strom.memcpy_ssd2ram(buf.address, fd, perm, CH)
            strom.memcpy_wait(r.dma_task_id)
            assert np.array_equal(buf.array[:64 * CH], _chunks(data, perm))
    finally:
        os.close(fd)


def test_ssd2ram_requires_dma_buffer(strom, rand_file):
    path, _ = rand_file(16 * CH)
    fd = _open(path)
    try:
        plain = np.zeros(16 * CH, dtype=np.uint8)
        with pytest.raises(strom.StromError) as e:
            strom.memcpy_ssd2ram(plain.ctypes.data, fd, np.arange(16, dtype=np.uint32), CH)
        assert e.value.errno == errno.EINVAL
    finally:
        os.close(fd)


def test_merge_rule_and_counters(strom, rand_file):
    strom.configure(max_request=128 << 10)
    path, data = rand_file(256 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(256 * CH) as buf:
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(256, dtype=np.uint32), CH)
            strom.memcpy_wait(r.dma_task_id)
            assert r.nr_ssd == 256 and r.nr_ram == 0
            # 2 MiB sequential in 128 KiB requests
            assert r.nr_dma_submit == (256 * CH) // (128 << 10)
            assert r.nr_dma_blocks == 256 * CH // 512
            assert r.avg_request_bytes == 128 << 10
            # reversed order: no two chunks are contiguous in both file and dest
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(255, -1, -1, dtype=np.uint32), CH)
            strom.memcpy_wait(r.dma_task_id)
            assert r.nr_dma_submit == 256
            assert np.array_equal(buf.array[:256 * CH], _chunks(data, range(255, -1, -1)))
    finally:
        os.close(fd)


def test_relseg_modulo(strom, rand_file):
    path, data = rand_file(32 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(8 * CH) as buf:
            ids = np.array([32, 33, 65, 3, 100, 0, 31, 64], dtype=np.uint32)
            r = strom.memcpy_ssd2ram(buf.address, fd, ids, CH, relseg_sz=32)
            strom.memcpy_wait(r.dma_task_id)
            assert np.array_equal(buf.array[:8 * CH], _chunks(data, ids, relseg=32))
    finally:
        os.close(fd)


def test_eof_rules(strom, rand_file):
    n = 10 * CH + 100            # last chunk partial
    path, data = rand_file(n)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(2 * CH) as buf:
            buf.array[:] = 0xAB
            r = strom.memcpy_ssd2ram(buf.address, fd, np.array([10], dtype=np.uint32), CH)
            strom.memcpy_wait(r.dma_task_id)
            assert np.array_equal(buf.array[:100], data[10 * CH:])
            assert (buf.array[100:CH] == 0).all()          # zero-filled past EOF
            # a chunk that starts at/after EOF is rejected (reference defect #10)
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_ssd2ram(buf.address, fd, np.array([11], dtype=np.uint32), CH)
            assert e.value.errno == errno.ERANGE
    finally:
        os.close(fd)


@pytest.mark.parametrize("chunk", [0, 1000, 4096 + 512])
def test_bad_chunk_size(strom, rand_file, chunk):
    path, _ = rand_file(16 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(16 * CH) as buf:
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_ssd2ram(buf.address, fd, np.arange(2, dtype=np.uint32), chunk)
            assert e.value.errno == errno.EINVAL
    finally:
        os.close(fd)


def _warm(path, chunk_ids, chunk=CH):
    fd = os.open(path, os.O_RDONLY)
    try:
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_RANDOM)      # no readahead
        for c in chunk_ids:
            os.pread(fd, chunk, c * chunk)
    finally:
        os.close(fd)


def test_ssd2gpu_page_cache_hybrid_reorder(strom, rand_file):
    """Cached chunks go to wb_buffer's tail (reverse order), storage chunks
    are packed at the head; chunk_ids is rewritten to the landing order."""
    nch = 32
    path, data = rand_file(nch * CH)
    cached = {3, 7, 8, 20, 31}
    _warm(path, cached)
    fd = _open(path)
    try:
        keep, hbm = _host_target(nch * CH)
        wb = np.zeros(nch * CH, dtype=np.uint8)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            ids = np.arange(nch, dtype=np.uint32)
            r = strom.memcpy_ssd2gpu(m.handle, 0, fd, ids, CH, wb_buffer=wb.ctypes.data)
            strom.memcpy_wait(r.dma_task_id)
            assert r.nr_ram == len(cached) and r.nr_ssd == nch - len(cached)
            ssd_ids = [i for i in range(nch) if i not in cached]
            assert list(ids[:r.nr_ssd]) == ssd_ids
            # RAM chunks fill from the tail: first cached chunk lands last
            assert list(ids[r.nr_ssd:]) == sorted(cached, reverse=True)
            assert np.array_equal(hbm[:r.nr_ssd * CH], _chunks(data, ssd_ids))
            tail = wb[r.nr_ssd * CH:]
            assert np.array_equal(tail, _chunks(data, ids[r.nr_ssd:]))
    finally:
        os.close(fd)


def test_pread_gpu_latency_probe(strom, rand_file):
    """Native QD1 probe: every read lands (last one checked) and is timed."""
    path, data = rand_file(64 * 4096)
    fd = _open(path)
    try:
        keep, hbm = _host_target(16 * 4096)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            offs = np.array([5, 17, 63, 0, 40], dtype=np.uint64) * 4096
            ns = strom.pread_gpu_latency(m.handle, 4096, fd, offs)
            assert ns.shape == (5,) and (ns > 0).all()
            assert np.array_equal(hbm[4096:8192], data[40 * 4096:41 * 4096])
            with pytest.raises(strom.StromError) as e:
                strom.pread_gpu_latency(m.handle, 0, fd, np.array([100], dtype=np.uint64) * 4096)
            assert e.value.errno == errno.ERANGE
    finally:
        os.close(fd)


def test_ssd2gpu_range_and_handle_checks(strom, rand_file):
    path, _ = rand_file(16 * CH)
    fd = _open(path)
    try:
        keep, hbm = _host_target(8 * CH)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_ssd2gpu(m.handle, CH, fd, np.arange(8, dtype=np.uint32), CH)
            assert e.value.errno == errno.ERANGE
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_ssd2gpu(m.handle + 999, 0, fd, np.arange(1, dtype=np.uint32), CH)
            assert e.value.errno == errno.ENOENT
    finally:
        os.close(fd)


def test_destination_offset_wrap_is_erange(strom, rand_file):
    """offset + bytes must not wrap past the mapping:
    both providers use the overflow-safe strom_core_check_range."""
    path, _ = rand_file(16 * CH)
    fd = _open(path)
    try:
        keep, hbm = _host_target(8 * CH)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            huge = (1 << 64) - 4096
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_ssd2gpu(m.handle, huge, fd, np.arange(2, dtype=np.uint32), CH)
            assert e.value.errno == errno.ERANGE
            with pytest.raises(strom.StromError) as e:
                strom.pread_gpu(m.handle, huge, fd, 0, 8192)
            assert e.value.errno == errno.ERANGE
            assert strom.pread_gpu(m.handle, 7 * CH, fd, 0, CH) == CH    # last slot fits
    finally:
        os.close(fd)


def test_gpu_registry_list_info_unmap(strom):
    keep, hbm = _host_target(300 * 1024)
    addr = hbm.ctypes.data + 4096                       # not 64 KiB aligned
    m = strom.map_gpu_memory(addr, 200 * 1024)
    try:
        assert m.gpu_page_sz == 65536
        info = strom.info_gpu_memory(m.handle)
        assert info["map_offset"] == 4096
        assert info["map_length"] == 4096 + 200 * 1024
        assert info["nitems"] == m.gpu_npages == 4
        assert info["paddrs"][0] == addr - 4096
        assert info["owner"] == os.geteuid()
        assert m.handle in strom.list_gpu_memory()
    finally:
        m.unmap()
    assert m.handle == 0
    with pytest.raises(strom.StromError) as e:
        strom.unmap_gpu_memory(12345)
    assert e.value.errno == errno.ENOENT


def test_wait_unknown_id(strom):
    with pytest.raises(strom.StromError) as e:
        strom.memcpy_wait(1 << 60)
    assert e.value.errno == errno.ENOENT


def test_fault_injection_reports_status(strom, rand_file):
    path, _ = rand_file(64 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(64 * CH) as buf:
            strom.configure(max_request=CH)                       # 1 request per chunk
            strom.fault_inject(fail_at=5, err=errno.EIO)
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(64, dtype=np.uint32), CH)
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_wait(r.dma_task_id)
            assert e.value.errno == errno.EIO and e.value.status == -errno.EIO
            # the failed record is consumed by WAIT: a second WAIT sees success
            strom.memcpy_wait(r.dma_task_id)
            # short read before EOF is an error too
            strom.fault_inject(short_at=3, short_bytes=512)
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(64, dtype=np.uint32), CH)
            with pytest.raises(strom.StromError):
                strom.memcpy_wait(r.dma_task_id)
    finally:
        os.close(fd)


def test_session_close_reclaims_failed_tasks(strom, rand_file):
    path, _ = rand_file(16 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(16 * CH) as buf:
            s = strom.Session()
            strom.fault_inject(fail_at=1)
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(16, dtype=np.uint32), CH, sess=s)
            # let it finish without waiting through the session
            import time
            deadline = time.time() + 5
            while strom.stat_info()["cur_dma_count"] and time.time() < deadline:
                time.sleep(0.01)
            time.sleep(0.05)
            assert s.close() == 1
            strom.fault_inject(0)
    finally:
        os.close(fd)


def test_timed_wait(strom, rand_file):
    path, _ = rand_file(16 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(16 * CH) as buf:
            strom.configure(max_request=CH)
            strom.fault_inject(delay_us=20000)                   # 20 ms per request
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(16, dtype=np.uint32), CH)
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_wait(r.dma_task_id, timeout=0.001)
            assert e.value.errno == errno.ETIME
            strom.memcpy_wait(r.dma_task_id, timeout=30)
    finally:
        strom.fault_inject(0)
        os.close(fd)


def test_check_file(strom, rand_file, tmp_path):
    path, _ = rand_file(4 * CH)
    fd = _open(path)
    try:
        info = strom.check_file(fd)
        assert info.support_dma64
    finally:
        os.close(fd)
    small = tmp_path / "small"
    small.write_bytes(b"x" * 100)                           # < PAGE_SIZE
    fd = _open(str(small))
    try:
        with pytest.raises(strom.StromError) as e:
            strom.check_file(fd)
        assert e.value.errno == errno.ENOTSUP
    finally:
        os.close(fd)
    wfd = os.open(path, os.O_WRONLY)
    try:
        with pytest.raises(strom.StromError) as e:
            strom.check_file(wfd)
        assert e.value.errno == errno.EBADF
    finally:
        os.close(wfd)


def test_stats_and_histograms(strom, rand_file):
    path, _ = rand_file(64 * CH)
    fd = _open(path)
    try:
        with strom.alloc_dma_buffer(64 * CH) as buf:
            strom.stat_hist(reset=True)
            before = strom.stat_info()
            r = strom.memcpy_ssd2ram(buf.address, fd, np.arange(64, dtype=np.uint32), CH)
            strom.memcpy_wait(r.dma_task_id)
            after = strom.stat_info()
            assert after["nr_ssd2gpu"] - before["nr_ssd2gpu"] == r.nr_dma_submit
            assert after["nr_submit_dma"] > before["nr_submit_dma"]
            h = strom.stat_hist()
            assert h["io_ns"].sum() >= r.nr_dma_submit
            assert h["task_ns"].sum() >= 1
            p50 = strom.hist_percentile(h["io_ns"], 50)
            assert 0 < p50 < 10e9
    finally:
        os.close(fd)


def test_concurrent_tasks_from_threads(strom, rand_file):
    import threading
    path, data = rand_file(128 * CH)
    fd = _open(path)
    errors = []
    try:
        with strom.alloc_dma_buffer(128 * CH) as buf:
            def worker(k):
                try:
                    ids = np.arange(k * 16, (k + 1) * 16, dtype=np.uint32)
                    s = strom.Session()
                    for _ in range(5):
                        r = strom.memcpy_ssd2ram(buf.address + k * 16 * CH, fd, ids, CH, sess=s)
                        strom.memcpy_wait(r.dma_task_id, sess=s)
                    s.close()
                except Exception as e:  # pragma: no cover
                    errors.append(e)
            ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
            [t.start() for t in ts]
            [t.join() for t in ts]
            assert not errors
            assert np.array_equal(buf.array[:128 * CH], data)
    finally:
        os.close(fd)


def test_pread_gpu_phase_probe(strom, rand_file):
    """Phase stamps of the synchronous path rise monotonically to the total,
    the data lands, and the raw O_DIRECT floor is measured alongside."""
    path, data = rand_file(64 * 4096)
    fd = _open(path)
    try:
        keep, hbm = _host_target(16 * 4096)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            offs = np.array([3, 9, 27, 50, 1], dtype=np.uint64) * 4096
            st = strom.pread_gpu_phases(m.handle, 0, fd, offs)
            assert st.shape == (5, len(strom.PHASES))
            for row in st:
                hit = row[row > 0].astype(np.int64)
                assert len(hit) >= 4 and (np.diff(hit) >= 0).all()
                assert row[-1] == hit.max()
            assert (st[:, strom.PHASES.index("storage")] > 0).all()
            assert np.array_equal(hbm[:4096], data[4096:8192])
            bd = strom.phase_breakdown(st)
            assert list(bd) == list(strom.PHASES) and bd["wait"] is not None
            raw = strom.pread_raw_latency(fd, offs)
            assert raw.shape == (5,) and (raw > 0).all()
            # interleaved pairs: the engine read of each pair lands its own
            # offset (offs[2i + 1]); the last one is in hbm
            pe, pr = strom.pread_pair_latency(m.handle, 0, fd, np.array([2, 7, 11, 4], dtype=np.uint64) * 4096)
            assert pe.shape == pr.shape == (2,) and (pe > 0).all() and (pr > 0).all()
            assert np.array_equal(hbm[:4096], data[4 * 4096:5 * 4096])
    finally:
        os.close(fd)


def test_coalesce_knob(strom):
    """Worker copy coalescing is a config key (default on), parsed as a bool."""
    assert strom.config_get("coalesce") == "1"
    strom.configure(coalesce=0)
    try:
        assert strom.config_get("coalesce") == "0"
    finally:
        strom.configure(coalesce=1)
    assert strom.config_get("coalesce") == "1"


def test_pread_gpu_per_thread_caches(strom, rand_file):
    """The synchronous path's per-thread mapping / file caches: an unmapped
    handle fails at once, a new mapping is seen, a descriptor number reused
    for another file reads the new file, and a file that grew is re-sized."""
    path, data = rand_file(16 * 4096)
    path2, data2 = rand_file(32 * 4096, seed=1, name="other.bin")
    keep, hbm = _host_target(4 * 4096)
    fd = _open(path)
    try:
        m = strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes)
        strom.pread_gpu_latency(m.handle, 0, fd, np.array([3 * 4096], dtype=np.uint64))
        assert np.array_equal(hbm[:4096], data[3 * 4096:4 * 4096])
        h = m.handle
        strom.unmap_gpu_memory(h)
        with pytest.raises(strom.StromError) as e:
            strom.pread_gpu_latency(h, 0, fd, np.array([0], dtype=np.uint64))
        assert e.value.errno == errno.ENOENT
        m = strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes)
        # the same descriptor number, another file
        fd2 = os.open(path2, os.O_RDONLY)
        os.dup2(fd2, fd)
        os.close(fd2)
        strom.pread_gpu_latency(m.handle, 4096, fd, np.array([20 * 4096], dtype=np.uint64))
        assert np.array_equal(hbm[4096:8192], data2[20 * 4096:21 * 4096])
        # the file grows: a read past the old size succeeds
        extra = np.random.default_rng(5).integers(0, 256, 8 * 4096, dtype=np.uint8)
        with open(path2, "ab") as f:
            f.write(extra.tobytes())
        strom.pread_gpu_latency(m.handle, 0, fd, np.array([33 * 4096], dtype=np.uint64))
        assert np.array_equal(hbm[:4096], extra[4096:8192])
        # ... and shrinks: past the new end is out of range, inside it reads
        os.truncate(path2, 10 * 4096)
        with pytest.raises(strom.StromError) as e:
            strom.pread_gpu_latency(m.handle, 0, fd, np.array([20 * 4096], dtype=np.uint64))
        assert e.value.errno == errno.ERANGE
        strom.pread_gpu_latency(m.handle, 0, fd, np.array([5 * 4096], dtype=np.uint64))
        assert np.array_equal(hbm[:4096], data2[5 * 4096:6 * 4096])
        strom.unmap_gpu_memory(m.handle)
    finally:
        os.close(fd)


def test_registered_file(strom, rand_file):
    """A registered file's id reads like its descriptor (pread_gpu, CHECK_FILE,
    SSD2GPU), keeps reading after the caller closes its descriptor and after
    the number is reused for another file, follows growth and shrinkage, and
    ends with unregister (-EBADF after)."""
    path, data = rand_file(16 * 4096)
    path2, data2 = rand_file(8 * 4096, seed=3, name="other.bin")
    keep, hbm = _host_target(4 * 4096)
    fd = _open(path)
    rf = strom.RegisteredFile(fd)
    assert rf.fd >= 0x7E000000
    with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
        strom.pread_gpu_latency(m.handle, 0, rf.fd, np.array([3 * 4096], dtype=np.uint64))
        assert np.array_equal(hbm[:4096], data[3 * 4096:4 * 4096])
        # the caller's descriptor closed, its number reused for another file
        os.close(fd)
        fd2 = os.open(path2, os.O_RDONLY)
        try:
            strom.pread_gpu_latency(m.handle, 4096, rf.fd, np.array([9 * 4096], dtype=np.uint64))
            assert np.array_equal(hbm[4096:8192], data[9 * 4096:10 * 4096])
            # the task path and CHECK_FILE take the id too
            ids = np.array([12, 13], dtype=np.uint32)
            wb = np.zeros(2 * 4096, dtype=np.uint8)
            t = strom.memcpy_ssd2gpu(m.handle, 0, rf.fd, ids, 4096, wb_buffer=wb.ctypes.data)
            strom.memcpy_wait(t.dma_task_id)
            for k, c in enumerate(ids.tolist()):
                got = hbm[k * 4096:(k + 1) * 4096] if k < t.nr_ssd else wb[k * 4096:(k + 1) * 4096]
                assert np.array_equal(got, data[c * 4096:(c + 1) * 4096])
            strom.check_file(rf.fd)
            pe, pr = strom.pread_pair_latency(m.handle, 0, rf.fd, np.array([2, 4], dtype=np.uint64) * 4096)
            assert (pe > 0).all() and (pr > 0).all()
            assert np.array_equal(hbm[:4096], data[4 * 4096:5 * 4096])
            # two ids, interleaved on one thread
            with strom.RegisteredFile(path2) as rf2:
                for k in (1, 7, 2):
                    strom.pread_gpu_latency(m.handle, 0, rf2.fd, np.array([k * 4096], dtype=np.uint64))
                    assert np.array_equal(hbm[:4096], data2[k * 4096:(k + 1) * 4096])
                    strom.pread_gpu_latency(m.handle, 0, rf.fd, np.array([k * 4096], dtype=np.uint64))
                    assert np.array_equal(hbm[:4096], data[k * 4096:(k + 1) * 4096])
            # growth: a read past the registered size re-reads it
            extra = np.random.default_rng(6).integers(0, 256, 4 * 4096, dtype=np.uint8)
            with open(path, "ab") as f:
                f.write(extra.tobytes())
            # ... and so does the task path (it planned with the
            # size cached at registration, -ERANGE past the old end)
            ids = np.array([16, 18], dtype=np.uint32)
            t = strom.memcpy_ssd2gpu(m.handle, 0, rf.fd, ids, 4096, wb_buffer=wb.ctypes.data)
            strom.memcpy_wait(t.dma_task_id)
            for k, c in enumerate(ids.tolist()):            # rewritten to the landing order
                got = hbm[k * 4096:(k + 1) * 4096] if k < t.nr_ssd else wb[k * 4096:(k + 1) * 4096]
                assert np.array_equal(got, extra[(c - 16) * 4096:(c - 15) * 4096])
            strom.pread_gpu_latency(m.handle, 0, rf.fd, np.array([17 * 4096], dtype=np.uint64))
            assert np.array_equal(hbm[:4096], extra[4096:8192])
            # shrinkage: past the new end is out of range
            os.truncate(path, 6 * 4096)
            with pytest.raises(strom.StromError) as e:
                strom.pread_gpu_latency(m.handle, 0, rf.fd, np.array([10 * 4096], dtype=np.uint64))
            assert e.value.errno == errno.ERANGE
            # the task path refuses at planning time, not with a late -EIO
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_ssd2gpu(m.handle, 0, rf.fd, np.array([8], dtype=np.uint32), 4096,
                                     wb_buffer=wb.ctypes.data)
            assert e.value.errno == errno.ERANGE
            strom.pread_gpu_latency(m.handle, 0, rf.fd, np.array([5 * 4096], dtype=np.uint64))
            assert np.array_equal(hbm[:4096], data[5 * 4096:6 * 4096])
            rf.close()
            with pytest.raises(strom.StromError) as e:
                strom.pread_gpu_latency(m.handle, 0, rf.fd if rf.fd >= 0 else 0x7E000000,
                                        np.array([0], dtype=np.uint64))
            assert e.value.errno == errno.EBADF
        finally:
            os.close(fd2)


def test_plain_descriptor_keeps_record_locks(strom, rand_file, tmp_path):
    """a thread alternating synchronous reads over two plain
    descriptors must not drop the process's fcntl record locks (closing ANY
    descriptor of a file releases them): by default no dup of the caller's
    descriptor is kept or closed.  A child process checks the lock."""
    import fcntl
    import subprocess
    import sys
    pa, _ = rand_file(8 * 4096)
    pb, _ = rand_file(8 * 4096, seed=2, name="b.bin")
    keep, hbm = _host_target(4096)
    fa, fb = _open(pa), _open(pb)
    lk = os.open(pa, os.O_RDWR)
    probe = ("import fcntl, os, sys\nfd = os.open(sys.argv[1], os.O_RDWR)\n"
             "try:\n    fcntl.lockf(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)\n    print('got')\n"
             "except OSError:\n    print('held')\n")
    try:
        fcntl.lockf(lk, fcntl.LOCK_EX)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            for k in range(4):
                for fd in (fa, fb, lk):
                    strom.pread_gpu_latency(m.handle, 0, fd, np.array([k * 4096], dtype=np.uint64))
        out = subprocess.run([sys.executable, "-c", probe, pa], capture_output=True, text=True,
                             timeout=60).stdout.strip()
        assert out == "held"
    finally:
        for fd in (fa, fb, lk):
            os.close(fd)
