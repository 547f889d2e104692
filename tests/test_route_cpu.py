"""Volume routes for the kernel provider from a (fake) sysfs tree: md raid0
zones/members and NVMe multipath paths (nvme_strom_amd/utils/route.py ->
STROM_IOCTL__SET_ROUTE, checked by kmod/strom_route.c).  The zones must remap
like the shared core's raid0 (kmod/strom_core.c), reference
kmod/nvme_strom.c:755-820."""
import ctypes as C
import os

import pytest

from nvme_strom_amd.utils import route as R


def _w(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text + "\n")


@pytest.fixture
def sysfs(tmp_path):
    s = str(tmp_path / "sys")
    # three NVMe members: nvme1n1 is a multipath head whose path is nvme1c3n1
    sizes = {"nvme0n1": 4 << 20, "nvme1n1": 4 << 20, "nvme2n1": 3 << 20}   # sectors
    for i, (d, n) in enumerate(sizes.items()):
        _w(f"{s}/block/{d}/dev", f"259:{i}")
        _w(f"{s}/block/{d}/size", str(n))
    os.makedirs(f"{s}/block/nvme1n1/multipath/nvme1c3n1")
    pci = f"{s}/devices/pci0000:40/0000:41:00.0"
    os.makedirs(pci)
    os.makedirs(f"{s}/class/nvme/nvme3")
    os.symlink(pci, f"{s}/class/nvme/nvme3/device")
    md = f"{s}/block/md0"
    _w(f"{md}/dev", "9:0")
    _w(f"{md}/md/level", "raid0")
    _w(f"{md}/md/chunk_size", str(64 << 10))
    for slot, d in enumerate(sizes):
        dd = f"{md}/md/dev-{d}"
        os.makedirs(dd)
        os.symlink(f"{s}/block/{d}", f"{dd}/block")
        _w(f"{dd}/slot", str(slot))
        _w(f"{dd}/offset", str(2048 * (slot + 1)))
        _w(f"{dd}/size", str(sizes[d] // 2 - 1024 * (slot + 1)))     # KiB, minus superblock
    return s


def test_raid0_route_zones_and_members(sysfs):
    r = R.route_for(sysfs, "md0")
    assert (r.major, r.minor, r.chunk_sects) == (9, 0, 128)
    assert [m.disk for m in r.members] == ["nvme0n1", "nvme1c3n1", "nvme2n1"]
    assert (r.members[0].major, r.members[0].minor) == (259, 0)
    assert r.members[1].major == 0 and r.members[1].name == "0000:41:00.0/nvme3/nvme1c3n1"
    assert [m.data_offset for m in r.members] == [2048, 4096, 6144]
    # member 2 is smallest: zone 0 stripes all three, zone 1 the larger two...
    assert [z["devs"] for z in r.zones][0] == [0, 1, 2]
    assert all(z["end"] > 0 for z in r.zones)
    ends = [z["end"] for z in r.zones]
    assert ends == sorted(ends)
    s = r.to_struct()
    assert C.sizeof(s) == 2648 and s.nmembers == 3 and s.nzones == len(r.zones)
    assert bytes(s.member_name[1]).rstrip(b"\0") == b"0000:41:00.0/nvme3/nvme1c3n1"


def test_route_zones_remap_like_the_core(sysfs):
    """Every stripe chunk of the array maps inside its member's data area,
    through the same core the kernel module uses (explicit zone members, as
    SET_ROUTE passes them)."""
    from nvme_strom_amd import _native as N
    from test_kmod_core_cpu import Raid0
    r = R.route_for(sysfs, "md0")
    g = Raid0(chunk_sects=r.chunk_sects, nzones=len(r.zones), ndisks=len(r.members))
    for z, zone in enumerate(r.zones):
        g.zone_end[z], g.zone_dev_start[z] = zone["end"], zone["dev_start"]
        g.zone_nb_dev[z] = len(zone["devs"])
        for k, d in enumerate(zone["devs"]):
            g.zone_devs[z][k] = d
    for i, m in enumerate(r.members):
        g.data_offset[i] = m.data_offset
    lib = N.lib()
    lib.strom_core_raid0_check.argtypes = [C.POINTER(Raid0)]
    lib.strom_core_raid0_map.argtypes = [C.POINTER(Raid0), C.c_uint64, C.c_uint32,
                                         C.POINTER(C.c_int), C.POINTER(C.c_uint64)]
    assert lib.strom_core_raid0_check(C.byref(g)) == 0
    mem, ms = C.c_int(), C.c_uint64()
    total = r.zones[-1]["end"]
    sizes = [4 << 20, 4 << 20, 3 << 20]
    used = set()
    for sector in range(0, total, 97 * r.chunk_sects + 8):
        sector -= sector % 8
        assert lib.strom_core_raid0_map(C.byref(g), sector, 8, C.byref(mem), C.byref(ms)) == 0
        assert ms.value + 8 <= sizes[mem.value], (sector, mem.value, ms.value)
        used.add(mem.value)
    assert used == {0, 1, 2}


def test_multipath_head_route(sysfs):
    r = R.route_for(sysfs, "nvme1n1")
    assert r.chunk_sects == 0 and len(r.members) == 1
    assert r.members[0].name == "0000:41:00.0/nvme3/nvme1c3n1"
    with pytest.raises(ValueError):
        R.route_for(sysfs, "nvme0n1")       # not a head, nothing to route


def test_route_cli_prints_json(sysfs, capsys):
    assert R.main(["--sysfs", sysfs, "md0"]) == 0
    out = capsys.readouterr().out
    assert '"volume": "md0"' in out and "nvme1c3n1" in out
