"""Stripe sets: one logical file over several member files (one per SSD),
striped in fixed units — native multi-SSD aggregation without md (SURVEY
§2.3 PAR2; the reference relies on md raid0, kmod/nvme_strom.c:755-820).

The mapping is checked against an independent model (byte-level
reassembly of the members), through SSD2RAM, SSD2GPU (host-emulated HBM)
and the streaming loader, with requests that must split at stripe edges.
"""
import errno
import os

import numpy as np
import pytest

CH = 8192


def _members(tmp_path, n, data, unit):
    import nvme_strom_amd as S
    paths = [str(tmp_path / f"m{k}.bin") for k in range(n)]
    size = S.write_striped(paths, data, unit)
    for p in paths:
        fd = os.open(p, os.O_RDONLY)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        os.close(fd)
    return paths, size


def _model(paths, unit, size):
    """Independent reassembly: read member files round-robin by unit."""
    blobs = [open(p, "rb").read() for p in paths]
    out, pos = bytearray(), [0] * len(paths)
    s = 0
    while len(out) < size:
        k = s % len(paths)
        out += blobs[k][pos[k]:pos[k] + unit]
        pos[k] += unit
        s += 1
    return np.frombuffer(bytes(out[:size]), dtype=np.uint8)


@pytest.mark.parametrize("n,unit", [(2, 64 << 10), (3, 16 << 10), (4, 1 << 20), (1, 8 << 10)])
def test_stripe_ssd2ram_matches_model(strom, tmp_path, n, unit):
    nbytes = 3 * n * unit + 5 * CH + 123          # partial tail stripe, partial chunk
    data = np.random.default_rng(n).integers(0, 256, nbytes, dtype=np.uint8)
    paths, size = _members(tmp_path, n, data, unit)
    assert np.array_equal(_model(paths, unit, size), data)
    nch = (size + CH - 1) // CH
    with strom.StripeSet(paths, unit) as ss, strom.alloc_dma_buffer(nch * CH) as buf:
        assert ss.size == size
        info = strom.check_file(ss.fd)
        assert info.support_dma64
        perm = np.random.default_rng(7).permutation(nch).astype(np.uint32)
        r = strom.memcpy_ssd2ram(buf.address, ss.fd, perm, CH)
        strom.memcpy_wait(r.dma_task_id)
        padded = np.zeros(nch * CH, dtype=np.uint8)
        padded[:size] = data
        exp = np.concatenate([padded[c * CH:(c + 1) * CH] for c in perm])
        assert np.array_equal(buf.array[:nch * CH], exp)
        # requests never cross into another member: at least one per unit
        if n > 1:
            assert r.nr_dma_submit >= min(nch, (size + unit - 1) // unit)


def test_stripe_ssd2gpu_and_pread(strom, tmp_path):
    n, unit = 4, 32 << 10
    data = np.random.default_rng(1).integers(0, 256, 40 * unit, dtype=np.uint8)
    paths, size = _members(tmp_path, n, data, unit)
    keep = np.zeros(size + 65536, dtype=np.uint8)
    off = (-keep.ctypes.data) % 65536
    hbm = keep[off:off + size]
    with strom.StripeSet(paths, unit) as ss, strom.map_gpu_memory(hbm.ctypes.data, size) as m:
        big = 64 << 10                                   # chunks spanning two stripes
        ids = np.arange(size // big, dtype=np.uint32)[::-1].copy()
        r = strom.memcpy_ssd2gpu(m.handle, 0, ss.fd, ids, big)
        strom.memcpy_wait(r.dma_task_id)
        exp = np.concatenate([data[c * big:(c + 1) * big] for c in ids])
        assert np.array_equal(hbm, exp)
        # the synchronous path (task-less for plain files) routes members too
        hbm[:] = 0
        assert strom.pread_gpu(m.handle, 4096, ss.fd, 3 * unit - 8192, 24576) == 24576
        assert np.array_equal(hbm[4096:4096 + 24576], data[3 * unit - 8192:3 * unit + 16384])


def test_stripe_stream_loader(strom, tmp_path):
    import torch
    from nvme_strom_amd.models.ssd2gpu_stream import StreamLoader
    from nvme_strom_amd.tensor import HbmBuffer
    n, unit = 3, 128 << 10
    data = np.random.default_rng(3).integers(0, 256, 8 << 20, dtype=np.uint8)
    paths, size = _members(tmp_path, n, data, unit)
    with strom.StripeSet(paths, unit) as ss:
        b = HbmBuffer(4 << 20, torch.device("cpu"))
        ld = StreamLoader(ss, segment_sz=1 << 20, chunk_sz=CH, buf=b, depth=3)
        ld.run(2 << 20, 4 << 20)
        assert np.array_equal(b.tensor.numpy(), data[2 << 20:6 << 20])
        ld.close()


def test_stripe_chunk_past_logical_end(strom, tmp_path):
    """A chunk that starts before the logical end and runs past it (and
    past the last stripe row) reads the tail as zeros, as for a file."""
    unit = 256 << 10
    data = np.random.default_rng(4).integers(0, 256, (6 << 20) + 12345, dtype=np.uint8)
    paths, size = _members(tmp_path, 3, data, unit)
    big = 1 << 20
    nch = (size + big - 1) // big
    keep = np.zeros(nch * big + 65536, dtype=np.uint8)
    off = (-keep.ctypes.data) % 65536
    hbm = keep[off:off + nch * big]
    hbm[:] = 0xEE
    with strom.StripeSet(paths, unit) as ss, strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
        r = strom.memcpy_ssd2gpu(m.handle, 0, ss.fd, np.arange(nch, dtype=np.uint32), big)
        strom.memcpy_wait(r.dma_task_id)
        assert np.array_equal(hbm[:size], data)
        assert not hbm[size:].any()


def test_stripe_validation(strom, tmp_path):
    unit = 16 << 10
    data = np.random.default_rng(0).integers(0, 256, 10 * unit, dtype=np.uint8)
    paths, size = _members(tmp_path, 2, data, unit)
    with pytest.raises(strom.StromError) as e:            # claims more than the members hold
        strom.StripeSet(paths, unit, size=size + unit)
    assert e.value.errno == errno.ERANGE
    with pytest.raises(strom.StromError) as e:
        strom.StripeSet(paths, 1000)                        # unit not a multiple of 4 KiB
    assert e.value.errno == errno.EINVAL
    ss = strom.StripeSet(paths, unit)
    fd = ss.fd
    ss.close()
    with strom.alloc_dma_buffer(CH) as buf:
        with pytest.raises(strom.StromError) as e:          # closed pseudo descriptor
            strom.memcpy_ssd2ram(buf.address, fd, np.arange(1, dtype=np.uint32), CH)
        assert e.value.errno == errno.EBADF
    # survives an engine reset (process-wide registry)
    with strom.StripeSet(paths, unit) as ss, strom.alloc_dma_buffer(2 * CH) as buf:
        strom.engine_reset()
        r = strom.memcpy_ssd2ram(buf.address, ss.fd, np.array([1, 0], dtype=np.uint32), CH)
        strom.memcpy_wait(r.dma_task_id)
        assert np.array_equal(buf.array[:2 * CH], np.concatenate([data[CH:2 * CH], data[:CH]]))
