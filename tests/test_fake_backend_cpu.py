"""The fake namespace backend (SURVEY §4 test strategy): reads served from a
file, completions delivered in a seeded random order.  Landing order,
chunk_ids rewriting, task refcounts, error propagation through WAIT and
staging reuse must not depend on completion order.
"""
import errno
import os
import threading

import numpy as np
import pytest

CH = 8192


@pytest.fixture
def fake(strom):
    strom.fake_backend(seed=12345)
    strom.configure(backend="fake", max_request=CH, queue_depth=16, workers=2)
    yield strom
    strom.configure(backend="uring", max_request=1 << 20, queue_depth=8, workers=4)


def _cat(data, ids):
    return np.concatenate([data[i * CH:(i + 1) * CH] for i in ids])


def test_fake_ssd2ram_out_of_order_completions(fake, rand_file):
    S = fake
    path, data = rand_file(256 * CH)
    fd = os.open(path, os.O_RDONLY)
    try:
        c0, r0 = S.fake_backend()
        with S.alloc_dma_buffer(256 * CH) as buf:
            perm = np.random.default_rng(5).permutation(256).astype(np.uint32)
            r = S.memcpy_ssd2ram(buf.address, fd, perm, CH)
            S.memcpy_wait(r.dma_task_id)
            assert np.array_equal(buf.array[:256 * CH], _cat(data, perm))
        c1, r1 = S.fake_backend()
        assert c1 - c0 >= 256 // 2          # one request per chunk (some merged)
        assert r1 - r0 > 0                  # and they really came back out of order
    finally:
        os.close(fd)


def test_fake_ssd2gpu_hybrid_landing(fake, rand_file):
    """Cached chunks to the write-back tail, storage chunks packed at the head
    in request order, whatever order their completions arrived in."""
    S = fake
    nch = 64
    path, data = rand_file(nch * CH)
    cached = {2, 9, 10, 33, 63}
    fdw = os.open(path, os.O_RDONLY)
    os.posix_fadvise(fdw, 0, 0, os.POSIX_FADV_RANDOM)      # no readahead around them
    for c in cached:
        os.pread(fdw, CH, c * CH)
    os.close(fdw)
    fd = os.open(path, os.O_RDONLY)
    try:
        keep = np.zeros(nch * CH + 65536, dtype=np.uint8)
        off = (-keep.ctypes.data) % 65536
        hbm = keep[off:off + nch * CH]
        wb = np.zeros(nch * CH, dtype=np.uint8)
        with S.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            ids = np.random.default_rng(2).permutation(nch).astype(np.uint32)
            req = ids.copy()
            r = S.memcpy_ssd2gpu(m.handle, 0, fd, ids, CH, wb_buffer=wb.ctypes.data)
            S.memcpy_wait(r.dma_task_id)
            assert r.nr_ram == len(cached)
            ssd = [int(i) for i in req if int(i) not in cached]
            assert list(ids[:r.nr_ssd]) == ssd
            assert np.array_equal(hbm[:r.nr_ssd * CH], _cat(data, ssd))
            assert np.array_equal(wb[r.nr_ssd * CH:], _cat(data, ids[r.nr_ssd:]))
    finally:
        os.close(fd)


def test_fake_error_mid_task_drains(fake, rand_file):
    S = fake
    path, data = rand_file(64 * CH)
    fd = os.open(path, os.O_RDONLY)
    try:
        with S.alloc_dma_buffer(64 * CH) as buf:
            S.fault_inject(fail_at=7, err=errno.EIO)
            r = S.memcpy_ssd2ram(buf.address, fd, np.arange(64, dtype=np.uint32), CH)
            with pytest.raises(S.StromError) as e:
                S.memcpy_wait(r.dma_task_id)
            assert e.value.errno == errno.EIO
            S.fault_inject(0)
            assert S.stat_info()["cur_dma_count"] == 0    # every request retired
            r = S.memcpy_ssd2ram(buf.address, fd, np.arange(64, dtype=np.uint32), CH)
            S.memcpy_wait(r.dma_task_id)
            assert np.array_equal(buf.array[:64 * CH], data)
    finally:
        S.fault_inject(0)
        os.close(fd)


def test_fake_concurrent_sessions(fake, rand_file):
    S = fake
    path, data = rand_file(128 * CH)
    fd = os.open(path, os.O_RDONLY)
    errors = []
    try:
        with S.alloc_dma_buffer(128 * CH) as buf:
            def worker(k):
                try:
                    s = S.Session()
                    ids = np.arange(k * 16, (k + 1) * 16, dtype=np.uint32)[::-1].copy()
                    for _ in range(4):
                        r = S.memcpy_ssd2ram(buf.address + k * 16 * CH, fd, ids, CH, sess=s)
                        S.memcpy_wait(r.dma_task_id, sess=s)
                    s.close()
                except Exception as e:  # pragma: no cover
                    errors.append(e)
            ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
            [t.start() for t in ts]
            [t.join() for t in ts]
            assert not errors
            exp = np.concatenate([_cat(data, list(range(k * 16, (k + 1) * 16))[::-1])
                                  for k in range(8)])
            assert np.array_equal(buf.array[:128 * CH], exp)
    finally:
        os.close(fd)
