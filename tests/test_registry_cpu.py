"""Registry lifecycle on the CPU: SSD2RAM destination lookup (address index,
VMA query for a caller's own mmap, stale-address rejection), DMA-buffer
garbage collection, and detaching a GPU mapping whose memory went away.

Reference semantics: SSD2RAM accepts only addresses inside a VMA of the
driver's DMA-buffer file (find_vma + f_op check, kmod/nvme_strom.c:1920-1946);
the nvidia free callback detaches a mapping whose GPU memory is freed
(kmod/pmemmap.c:150-208).
"""
import ctypes as C
import errno
import mmap
import os

import numpy as np
import pytest

CH = 8192

_libc = C.CDLL(None, use_errno=True)
_libc.mmap.restype = C.c_void_p
_libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
_libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
MAP_FIXED_NOREPLACE = 0x100000


def _anon(n, at=None):
    flags = mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS | (MAP_FIXED_NOREPLACE if at else 0)
    p = _libc.mmap(at, n, mmap.PROT_READ | mmap.PROT_WRITE, flags, -1, 0)
    assert p not in (None, C.c_void_p(-1).value), os.strerror(C.get_errno())
    return p


def test_ssd2ram_engine_mapping_and_foreign_mmap(strom, rand_file):
    path, data = rand_file(32 * CH)
    fd = os.open(path, os.O_RDONLY)
    try:
        with strom.alloc_dma_buffer(32 * CH) as buf:
            ids = np.arange(32, dtype=np.uint32)
            r = strom.memcpy_ssd2ram(buf.address, fd, ids, CH)
            strom.memcpy_wait(r.dma_task_id)
            assert np.array_equal(buf.array[:32 * CH], data)
            # the caller's own mapping of the same fd, at an offset: found by
            # the VMA query, offset = vm_pgoff + (addr - vm_start)
            own = mmap.mmap(buf.fd, buf.length, flags=mmap.MAP_SHARED,
                            prot=mmap.PROT_READ | mmap.PROT_WRITE)
            try:
                view = np.frombuffer(own, dtype=np.uint8)
                addr = view.ctypes.data + 4 * CH
                r = strom.memcpy_ssd2ram(addr, fd, np.array([7, 3], dtype=np.uint32), CH)
                strom.memcpy_wait(r.dma_task_id)
                assert np.array_equal(view[4 * CH:6 * CH], _cat(data, [7, 3]))
                # same bytes through the engine's mapping (one memfd)
                assert np.array_equal(buf.array[4 * CH:6 * CH], _cat(data, [7, 3]))
                # a range running past the end of the mapping
                with pytest.raises(strom.StromError) as e:
                    strom.memcpy_ssd2ram(view.ctypes.data + buf.length - CH, fd,
                                         np.array([0, 1], dtype=np.uint32), CH)
                assert e.value.errno == errno.EINVAL
                del view
            finally:
                own.close()
    finally:
        os.close(fd)


def _cat(data, ids):
    return np.concatenate([data[i * CH:(i + 1) * CH] for i in ids])


def test_ssd2ram_rejects_stale_address(strom, rand_file):
    """After the buffer is unmapped and something else is mapped at the same
    address, SSD2RAM must refuse it instead of writing there."""
    path, _ = rand_file(16 * CH)
    fd = os.open(path, os.O_RDONLY)
    try:
        buf = strom.alloc_dma_buffer(16 * CH)
        addr, length = buf.address, buf.length
        buf.close()
        with pytest.raises(strom.StromError) as e:      # nothing mapped there
            strom.memcpy_ssd2ram(addr, fd, np.arange(4, dtype=np.uint32), CH)
        assert e.value.errno == errno.EINVAL
        p = _anon(length, at=addr)                      # reuse of the address
        try:
            assert p == addr
            with pytest.raises(strom.StromError) as e:
                strom.memcpy_ssd2ram(addr, fd, np.arange(4, dtype=np.uint32), CH)
            assert e.value.errno == errno.EINVAL
        finally:
            _libc.munmap(p, length)
    finally:
        os.close(fd)


def test_dmabuf_gc_drops_released_buffers(strom):
    base = strom.dmabuf_gc()
    bufs = [strom.alloc_dma_buffer(1 << 20) for _ in range(3)]
    assert strom.dmabuf_gc() == base + 3
    # fd closed but still mapped by the caller: stays registered
    own = mmap.mmap(bufs[0].fd, bufs[0].length, flags=mmap.MAP_SHARED)
    for b in bufs:
        b.close()
    assert strom.dmabuf_gc() == base + 1
    own.close()
    assert strom.dmabuf_gc() == base


def test_ssd2gpu_detaches_freed_range(strom, rand_file):
    """Emulated HBM that is unmapped after MAP: the next SSD2GPU / pread
    fails with ENOENT and the handle disappears from LIST."""
    path, _ = rand_file(16 * CH)
    fd = os.open(path, os.O_RDONLY)
    n = 8 * CH
    p = _anon(n)
    try:
        before = strom.gpu_detached()
        m = strom.map_gpu_memory(p, n)
        r = strom.memcpy_ssd2gpu(m.handle, 0, fd, np.arange(2, dtype=np.uint32), CH)
        strom.memcpy_wait(r.dma_task_id)
        _libc.munmap(p, n)
        p = None
        with pytest.raises(strom.StromError) as e:
            strom.memcpy_ssd2gpu(m.handle, 0, fd, np.arange(2, dtype=np.uint32), CH)
        assert e.value.errno == errno.ENOENT
        assert strom.gpu_detached() == before + 1
        assert m.handle not in strom.list_gpu_memory()
        with pytest.raises(strom.StromError) as e:
            strom.pread_gpu(m.handle, 0, fd, 0, 4096)
        assert e.value.errno == errno.ENOENT
        m.handle = 0                                    # already gone
    finally:
        if p:
            _libc.munmap(p, n)
        os.close(fd)


def test_check_freed_knob(strom, rand_file):
    path, _ = rand_file(4 * CH)
    fd = os.open(path, os.O_RDONLY)
    n = 4 * CH
    p = _anon(n)
    try:
        strom.configure(reset=False, check_freed=0)
        m = strom.map_gpu_memory(p, n)
        # the range is still mapped: works with or without the check
        r = strom.memcpy_ssd2gpu(m.handle, 0, fd, np.arange(1, dtype=np.uint32), CH)
        strom.memcpy_wait(r.dma_task_id)
        m.unmap()
    finally:
        strom.configure(reset=False, check_freed=1)
        _libc.munmap(p, n)
        os.close(fd)
