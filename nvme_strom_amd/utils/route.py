"""Volume routes for the kernel provider: md raid0 arrays and NVMe multipath
heads described from sysfs as ``STROM_IOCTL__SET_ROUTE`` arguments.

The reference module read md/raid0 and nvme internals directly through
vendored private headers (kmod/nvme_strom.c:185-367, :755-820,
kmod/514.6.2.el7/).  The MI355X module uses exported kernel interfaces only,
so the admin registers what it cannot see (kmod/strom_route.c):

  * md raid0 ``mdX``: chunk size, zones (members grouped by size, as
    drivers/md/raid0.c create_strip_zones builds them), per-member data
    offset, and the member namespaces;
  * a multipath head ``nvmeXnY`` (or a raid0 member that is one): the hidden
    path disk ``nvmeXcZnY`` to submit on, named ``<pci>/<ctrl>/<disk>``
    because a hidden disk has no openable dev_t.

``python -m nvme_strom_amd.utils.route [--sysfs /sys] [--apply] md0 nvme1n1``
prints the routes (JSON) and, with ``--apply`` under the kernel provider,
registers them (needs CAP_SYS_ADMIN).  ``sysfs`` is a parameter so the CPU
tests can run it against a fake tree.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
from dataclasses import dataclass, field
from typing import List, Optional

MAX_ZONES = 16
MAX_DISKS = 32
SET_ROUTE = 0x5387          # _IO('S', 0x87)


class SetRoute(C.Structure):
    """struct strom_set_route (csrc/include/strom/uapi.h), 2648 bytes."""
    _fields_ = [("volume_major", C.c_uint32), ("volume_minor", C.c_uint32),
                ("nmembers", C.c_uint32), ("chunk_sects", C.c_uint32),
                ("nzones", C.c_uint32), ("reserved", C.c_uint32),
                ("zone_end", C.c_uint64 * MAX_ZONES), ("zone_dev_start", C.c_uint64 * MAX_ZONES),
                ("zone_nb_dev", C.c_uint32 * MAX_ZONES),
                ("zone_devs", (C.c_uint8 * MAX_DISKS) * MAX_ZONES),
                ("member_major", C.c_uint32 * MAX_DISKS), ("member_minor", C.c_uint32 * MAX_DISKS),
                ("data_offset", C.c_uint64 * MAX_DISKS),
                ("member_name", (C.c_char * 40) * MAX_DISKS)]


assert C.sizeof(SetRoute) == 2648


@dataclass
class Member:
    disk: str                     # the namespace disk (or a path disk)
    major: int = 0
    minor: int = 0
    name: str = ""                # "<pci>/<ctrl>/<path disk>" for hidden paths
    sectors: int = 0
    data_offset: int = 0


@dataclass
class Route:
    volume: str
    major: int
    minor: int
    chunk_sects: int = 0          # 0: single-path alias
    zones: List[dict] = field(default_factory=list)   # {end, dev_start, devs}
    members: List[Member] = field(default_factory=list)

    def to_struct(self) -> SetRoute:
        r = SetRoute(volume_major=self.major, volume_minor=self.minor,
                     nmembers=len(self.members), chunk_sects=self.chunk_sects,
                     nzones=len(self.zones))
        for z, zone in enumerate(self.zones):
            r.zone_end[z] = zone["end"]
            r.zone_dev_start[z] = zone["dev_start"]
            r.zone_nb_dev[z] = len(zone["devs"])
            for k, d in enumerate(zone["devs"]):
                r.zone_devs[z][k] = d
        for i, m in enumerate(self.members):
            r.member_major[i], r.member_minor[i] = m.major, m.minor
            r.data_offset[i] = m.data_offset
            r.member_name[i].value = m.name.encode()
        return r

    def as_dict(self) -> dict:
        return dict(volume=self.volume, dev=f"{self.major}:{self.minor}",
                    chunk_sects=self.chunk_sects, zones=self.zones,
                    members=[m.__dict__ for m in self.members])


def _read(path: str, default: Optional[str] = None) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def _devt(sysfs: str, disk: str):
    v = _read(os.path.join(sysfs, "block", disk, "dev"))
    if not v:
        raise FileNotFoundError(f"{disk}: no dev in sysfs")
    ma, mi = v.split(":")
    return int(ma), int(mi)


def _path_member(sysfs: str, head: str) -> Optional[Member]:
    """First path of a multipath head, named <pci>/<ctrl>/<path disk>."""
    mp = os.path.join(sysfs, "block", head, "multipath")
    if not os.path.isdir(mp):
        return None
    paths = sorted(os.listdir(mp))
    if not paths:
        return None
    path = paths[0]                               # nvme<subsys>c<ctrl>n<ns>
    ctrl = "nvme" + path.split("c", 1)[1].split("n", 1)[0]
    dev = os.path.realpath(os.path.join(sysfs, "class", "nvme", ctrl, "device"))
    pci = os.path.basename(dev)
    return Member(disk=path, name=f"{pci}/{ctrl}/{path}")


def _member(sysfs: str, disk: str) -> Member:
    m = _path_member(sysfs, disk)
    if m is None:
        ma, mi = _devt(sysfs, disk)
        m = Member(disk=disk, major=ma, minor=mi)
    m.sectors = int(_read(os.path.join(sysfs, "block", disk, "size"), "0"))
    return m


def raid0_route(sysfs: str, md: str) -> Route:
    base = os.path.join(sysfs, "block", md, "md")
    if _read(os.path.join(base, "level")) != "raid0":
        raise ValueError(f"{md} is not raid0")
    chunk = int(_read(os.path.join(base, "chunk_size"), "0")) >> 9
    if chunk < 8 or chunk % 8:
        raise ValueError(f"{md}: chunk of {chunk} sectors is not a multiple of 4 KiB")
    mem = []
    for e in os.listdir(base):
        if not e.startswith("dev-"):
            continue
        dd = os.path.join(base, e)
        disk = os.path.basename(os.path.realpath(os.path.join(dd, "block")))
        slot = int(_read(os.path.join(dd, "slot"), str(len(mem))))
        off = int(_read(os.path.join(dd, "offset"), "0"))
        size = int(_read(os.path.join(dd, "size"), "0")) * 2        # KiB -> sectors
        mem.append((slot, disk, off, size))
    mem.sort()
    if not mem or len(mem) > MAX_DISKS:
        raise ValueError(f"{md}: {len(mem)} members")
    ma, mi = _devt(sysfs, md)
    r = Route(volume=md, major=ma, minor=mi, chunk_sects=chunk)
    for _, disk, off, _size in mem:
        m = _member(sysfs, disk)
        m.data_offset = off
        r.members.append(m)
    # zones: distinct member sizes rounded down to the chunk (raid0.c)
    sizes = [s // chunk * chunk for _, _, _, s in mem]
    prev = end = 0
    for sz in sorted(set(sizes)):
        if sz == prev:
            continue
        devs = [i for i, s in enumerate(sizes) if s >= sz]
        end += (sz - prev) * len(devs)
        r.zones.append(dict(end=end, dev_start=prev, devs=devs))
        prev = sz
    if len(r.zones) > MAX_ZONES:
        raise ValueError(f"{md}: {len(r.zones)} zones")
    return r


def head_route(sysfs: str, head: str) -> Route:
    m = _path_member(sysfs, head)
    if m is None:
        raise ValueError(f"{head} is not a multipath head")
    ma, mi = _devt(sysfs, head)
    m.sectors = int(_read(os.path.join(sysfs, "block", head, "size"), "0"))
    return Route(volume=head, major=ma, minor=mi, members=[m])


def route_for(sysfs: str, volume: str) -> Route:
    volume = os.path.basename(volume)
    if os.path.isdir(os.path.join(sysfs, "block", volume, "md")):
        return raid0_route(sysfs, volume)
    return head_route(sysfs, volume)


def apply(route: Route) -> None:
    from .. import api
    if api.provider() != "kernel":
        raise RuntimeError("routes are for the kernel provider (/dev/nvme-strom); the userspace "
                           "engine reads md and multipath volumes through the block layer")
    arg = route.to_struct()
    api.session().ioctl(SET_ROUTE, arg, "SET_ROUTE")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("volumes", nargs="+")
    ap.add_argument("--sysfs", default="/sys")
    ap.add_argument("--apply", action="store_true")
    a = ap.parse_args(argv)
    routes = [route_for(a.sysfs, v) for v in a.volumes]
    print(json.dumps([r.as_dict() for r in routes], indent=1))
    if a.apply:
        for r in routes:
            apply(r)
    return 0


if __name__ == "__main__":
    sys.exit(main())
