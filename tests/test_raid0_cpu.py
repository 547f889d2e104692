"""md RAID-0 remap (reference kmod/nvme_strom.c:733-820) against an
independent model of raid0 zones: zone z spans md sectors
[zone_end[z-1], zone_end[z]) striped in chunk_sects units over the members
still present in that zone."""
import ctypes as C
import errno

import numpy as np
import pytest

from nvme_strom_amd import _native as N


def model(zones, chunk, offsets, sector, nr):
    """zones: list of (end, dev_start, members)."""
    start = 0
    for end, dev_start, members in zones:
        if sector < end:
            break
        start = end
    else:
        return -errno.ERANGE, None, None
    if sector % chunk + nr > chunk:
        return -errno.ESPIPE, None, None
    rel = sector - start
    chunk_no, in_chunk = divmod(rel, chunk)
    row, col = divmod(chunk_no, len(members))
    m = members[col]
    return 0, m, dev_start + row * chunk + in_chunk + offsets[m]


def native(zones, chunk, offsets, sector, nr, disks):
    ze = (C.c_uint64 * len(zones))(*[z[0] for z in zones])
    zs = (C.c_uint64 * len(zones))(*[z[1] for z in zones])
    zn = (C.c_int * len(zones))(*[len(z[2]) for z in zones])
    off = (C.c_uint64 * disks)(*offsets)
    mem, ms = C.c_int(), C.c_uint64()
    rc = N.lib().strom_raid0_map(ze, zs, zn, len(zones), chunk, off, disks, sector, nr,
                                 C.byref(mem), C.byref(ms))
    return rc, (mem.value if rc == 0 else None), (ms.value if rc == 0 else None)


@pytest.mark.parametrize("disks,chunk", [(2, 128), (4, 1024), (3, 256)])
def test_single_zone(disks, chunk):
    per = 100 * chunk
    zones = [(per * disks, 0, list(range(disks)))]
    offsets = [2048 * (i + 1) for i in range(disks)]
    rng = np.random.default_rng(disks)
    for _ in range(2000):
        s = int(rng.integers(0, per * disks))
        nr = int(rng.integers(1, 17))
        assert native(zones, chunk, offsets, s, nr, disks) == model(zones, chunk, offsets, s, nr)


def test_multi_zone_uneven_members():
    # members 0,1 are larger: zone 0 stripes over 3 disks, zone 1 over the last 2
    chunk = 128
    zones = [(3 * 1000 * chunk, 0, [0, 1, 2]), (3 * 1000 * chunk + 2 * 500 * chunk, 1000 * chunk, [1, 2])]
    offsets = [0, 8, 16]
    rng = np.random.default_rng(0)
    for _ in range(3000):
        s = int(rng.integers(0, zones[-1][0] + 100))
        nr = int(rng.integers(1, 9))
        assert native(zones, chunk, offsets, s, nr, 3) == model(zones, chunk, offsets, s, nr)


def test_chunk_crossing_rejected():
    zones = [(4 * 64 * 10, 0, [0, 1, 2, 3])]
    rc, _, _ = native(zones, 64, [0] * 4, 60, 8, 4)
    assert rc == -errno.ESPIPE
