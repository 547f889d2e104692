"""MEMCPY_SSD2GPU_EXTENTS: exact byte-range reads for an
Arrow scan's column buffers instead of fixed chunk ids.  The layout (runs
of page-widened extents, holes up to gap_max read through, runs back to
back) is checked against an independent Python model, the data against the
file, the byte accounting (bytes_read = extents + gap_bytes) and the
request sizes against max_request; errors for unsorted / overlapping /
past-EOF extents and a too-small destination; a stripe set takes them too.
The shared core (kmod/strom_core.c strom_core_plan_xfer) is the kernel
provider's planner as well."""
import errno
import os

import numpy as np
import pytest

PAGE = 4096


def _host_target(nbytes):
    buf = np.zeros(nbytes + 65536, dtype=np.uint8)
    off = (-buf.ctypes.data) % 65536
    return buf, buf[off:off + nbytes]


def model_layout(offs, lens, gap, isize):
    """(dst offsets, dst span, bytes read) the planner must produce."""
    runs, dst, cur = [], [], None
    for o, n in zip(offs, lens):
        if n == 0:
            dst.append(0)
            continue
        a, b = o // PAGE * PAGE, -(-(o + n) // PAGE) * PAGE
        if cur is not None and a <= cur[1] + gap:
            cur[1] = max(cur[1], b)
        else:
            d = cur[2] + cur[1] - cur[0] if cur is not None else 0
            cur = [a, b, d]
            runs.append(cur)
        dst.append(cur[2] + o - cur[0])
    span = cur[2] + cur[1] - cur[0] if cur is not None else 0
    eof = -(-isize // PAGE) * PAGE
    read = sum(max(0, min(b, eof) - a) for a, b, _ in runs)
    return np.array(dst, dtype=np.uint64), span, read


def _random_extents(rng, size, n):
    """Sorted, disjoint byte ranges with gaps from 0 to ~300 KiB, 8-byte
    aligned like Arrow buffers (some unaligned), some empty."""
    offs, lens = [], []
    pos = int(rng.integers(0, 5000))
    while len(offs) < n and pos < size - 16:
        ln = int(rng.choice([0, int(rng.integers(1, 64)), int(rng.integers(1, 200_000))]))
        ln = min(ln, size - pos)
        offs.append(pos)
        lens.append(ln)
        gap = int(rng.choice([0, 8, int(rng.integers(1, 9000)), int(rng.integers(9000, 300_000))]))
        pos += ln + gap
        if rng.random() < 0.7:
            pos = (pos + 7) & ~7
    return np.array(offs, np.uint64), np.array(lens, np.uint64)


@pytest.mark.parametrize("gap", [0, 8192, 65536, 1 << 20])
def test_extents_layout_data_and_accounting(strom, rand_file, gap):
    size = 6 << 20
    path, data = rand_file(size + 1234, seed=9)        # a tail past the last page
    rng = np.random.default_rng(gap + 1)
    offs, lens = _random_extents(rng, size + 1234, 300)
    want_dst, span, read = model_layout(offs.tolist(), lens.tolist(), gap, size + 1234)
    x = strom.extents_array(offs, lens)
    fd = os.open(path, os.O_RDONLY)
    try:
        plan = strom.memcpy_ssd2gpu_extents(0, 0, fd, x, gap_max=gap, plan_only=True)
        assert np.array_equal(plan.dst_off, want_dst)
        assert plan.dst_bytes == span and plan.bytes_read == read
        assert plan.bytes_read == int(lens.sum()) + plan.gap_bytes
        keep, hbm = _host_target(span + 8192)
        hbm[:] = 0xEE
        x2 = strom.extents_array(offs, lens)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            r = strom.memcpy_ssd2gpu_extents(m.handle, 4096, fd, x2, gap_max=gap)
            strom.memcpy_wait(r.dma_task_id)
        assert np.array_equal(r.dst_off, want_dst) and r.bytes_read == read
        for o, n, d in zip(offs.tolist(), lens.tolist(), r.dst_off.tolist()):
            if n:
                assert np.array_equal(hbm[4096 + d:4096 + d + n], data[o:o + n]), (o, n, d)
        assert hbm[4096 + span:].max() == 0xEE and hbm[:4096].max() == 0xEE
        # requests: merged up to max_request, the sectors are the bytes read
        mreq = int(strom.config_get("max_request"))
        assert r.nr_dma_submit >= -(-read // mreq)
        assert r.nr_dma_blocks * 512 == read
    finally:
        os.close(fd)


def test_extents_merge_count_follows_gap(strom, rand_file):
    """Holes at most gap_max are read through (fewer, longer requests);
    larger holes start a new run."""
    path, _ = rand_file(8 << 20, seed=2)
    offs = np.arange(0, 8 << 20, 256 << 10, dtype=np.uint64)      # 32 KiB every 256 KiB
    lens = np.full(len(offs), 32 << 10, np.uint64)
    fd = os.open(path, os.O_RDONLY)
    try:
        tight = strom.memcpy_ssd2gpu_extents(0, 0, fd, strom.extents_array(offs, lens),
                                             gap_max=0, plan_only=True)
        loose = strom.memcpy_ssd2gpu_extents(0, 0, fd, strom.extents_array(offs, lens),
                                             gap_max=256 << 10, plan_only=True)
    finally:
        os.close(fd)
    assert tight.gap_bytes == 0 and tight.dst_bytes == int(lens.sum())
    assert loose.gap_bytes == len(offs) * (224 << 10) - (224 << 10)
    assert loose.dst_bytes == loose.bytes_read == (8 << 20) - (224 << 10)


def test_extents_errors(strom, rand_file):
    path, _ = rand_file(1 << 20, seed=4)
    keep, hbm = _host_target(256 << 10)
    fd = os.open(path, os.O_RDONLY)
    try:
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            cases = [
                ([8192, 0], [100, 100], errno.EINVAL),            # unsorted
                ([0, 50], [100, 100], errno.EINVAL),              # overlapping
                ([(1 << 20) - 10], [100], errno.ERANGE),          # past EOF
                ([0], [512 << 10], errno.ERANGE),                 # destination too small
            ]
            for o, n, err in cases:
                with pytest.raises(strom.StromError) as e:
                    strom.memcpy_ssd2gpu_extents(m.handle, 0, fd, strom.extents_array(o, n))
                assert e.value.errno == err, (o, n)
            # nothing to read: a task that completes at once
            r = strom.memcpy_ssd2gpu_extents(m.handle, 0, fd, strom.extents_array([5], [0]))
            strom.memcpy_wait(r.dma_task_id)
            assert r.bytes_read == 0 and r.dst_bytes == 0
    finally:
        os.close(fd)


def test_extents_on_a_stripe_set(strom, tmp_path):
    """A stripe set's members serve the extents (the planner splits runs at
    stripe boundaries)."""
    unit, n = 64 << 10, 3
    rng = np.random.default_rng(7)
    logical = rng.integers(0, 256, 2 << 20, dtype=np.uint8)
    paths = []
    for k in range(n):
        stripes = [logical[s * unit:(s + 1) * unit] for s in range(k, len(logical) // unit, n)]
        p = str(tmp_path / f"m{k}")
        np.concatenate(stripes).tofile(p)
        paths.append(p)
    fds = [os.open(p, os.O_RDONLY) for p in paths]
    try:
        ss = strom.StripeSet(fds, unit, len(logical))
        offs = np.array([100, 70_000, 300_000, 1_000_000], np.uint64)
        lens = np.array([5000, 200_000, 8, 900_000], np.uint64)
        x = strom.extents_array(offs, lens)
        plan = strom.memcpy_ssd2gpu_extents(0, 0, ss.fd, strom.extents_array(offs, lens),
                                            gap_max=16384, plan_only=True)
        keep, hbm = _host_target(plan.dst_bytes)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            r = strom.memcpy_ssd2gpu_extents(m.handle, 0, ss.fd, x, gap_max=16384)
            strom.memcpy_wait(r.dma_task_id)
        for o, ln, d in zip(offs.tolist(), lens.tolist(), r.dst_off.tolist()):
            assert np.array_equal(hbm[d:d + ln], logical[o:o + ln])
        ss.close()
    finally:
        for fd in fds:
            os.close(fd)


@pytest.mark.parametrize("codec", ["zstd", "lz4"])
def test_arrow_scan_groups_read_as_extents(strom, tmp_path, codec):
    """An Arrow scan's groups (ArrowScan.EXTENTS): the group's buffers read
    through MEMCPY_SSD2GPU_EXTENTS into (host-emulated) HBM land where the
    launch tables point — every raw buffer pointer and decoder source is an
    extent's slot offset holding the file's bytes — and the group reads its
    buffers' bytes plus the reported gap bytes, nothing else."""
    pa = pytest.importorskip("pyarrow")
    import arrowgen
    from nvme_strom_amd.models.arrow_scan import ArrowScan
    from nvme_strom_amd.ops import decompress as D
    path = str(tmp_path / f"t_{codec}.arrow")
    arrowgen.write(path, arrowgen.table(6000, seed=3), compression=codec, batch_rows=500)
    raw = np.fromfile(path, dtype=np.uint8)
    sc = ArrowScan(path, "cpu")
    assert sc.EXTENTS
    names = ["i64", "s", "f64", "dec"]
    plan, cols, rows = sc._plan(names)
    groups = sc._groups(plan)
    fd = os.open(path, os.O_RDONLY)
    try:
        for g in groups:
            ext = g.ext
            keep, hbm = _host_target(g.span + 4096)
            x = ext.copy()
            with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
                r = strom.memcpy_ssd2gpu_extents(m.handle, 0, fd, x, gap_max=sc.EXTENT_GAP)
                strom.memcpy_wait(r.dma_task_id)
            assert np.array_equal(x["dst_off"], ext["dst_off"])
            assert r.bytes_read == int(ext["len"].sum()) + r.gap_bytes == g.read_bytes
            for o, n, d in zip(ext["file_off"].tolist(), ext["len"].tolist(),
                               ext["dst_off"].tolist()):
                assert np.array_equal(hbm[d:d + n], raw[o:o + n])
            starts = set(ext["dst_off"].tolist())
            assert set(g.ptr_rel[g.ptr_kind == 1].tolist()) <= starts
            for dsc in (g.descs, g.descs_lanes):
                if dsc is not None:
                    assert set(dsc[D.DESC_DTYPE.names[0]].tolist()) <= starts
    finally:
        os.close(fd)
        sc.close()


@pytest.mark.parametrize("gap", [0, 65536])
def test_probe_request_model_matches_planner(strom, rand_file, gap):
    """tools/arrow_read_probe.requests() — the raw comparator's request list
    — issues the planner's requests: same count, same bytes."""
    from types import SimpleNamespace
    from nvme_strom_amd.tools.arrow_read_probe import requests
    size = 8 << 20
    path, _ = rand_file(size, seed=5)
    rng = np.random.default_rng(gap + 7)
    offs, lens = _random_extents(rng, size - (1 << 20), 200)
    x = strom.extents_array(offs, lens)
    mreq = int(strom.config_get("max_request"))
    fd = os.open(path, os.O_RDONLY)
    try:
        plan = strom.memcpy_ssd2gpu_extents(0, 0, fd, x, gap_max=gap, plan_only=True)
        keep, hbm = _host_target(plan.dst_bytes)
        with strom.map_gpu_memory(hbm.ctypes.data, hbm.nbytes) as m:
            r = strom.memcpy_ssd2gpu_extents(m.handle, 0, fd, strom.extents_array(offs, lens),
                                             gap_max=gap)
            strom.memcpy_wait(r.dma_task_id)
    finally:
        os.close(fd)
    ro, rl = requests([SimpleNamespace(ext=x)], gap, mreq)
    assert len(ro) == r.nr_dma_submit
    assert int(rl.astype(np.int64).sum()) == r.bytes_read == r.nr_dma_blocks * 512
    assert (np.diff(ro.astype(np.int64)) > 0).all() and int(rl.max()) <= mreq
