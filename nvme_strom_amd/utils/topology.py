"""PCIe topology: which NVMe controllers sit near which GPU.

The reference picks one GPU by index and never asks where the SSD is
(utils/nvme_test.c:800-832; CHECK_FILE reports only a NUMA node,
kmod/nvme_strom.c:249-261).  Peer-to-peer NVMe -> HBM traffic is cheapest
when the SSD and the GPU share a PCIe switch (the TLPs turn around below the
root port), then a root port, then a host bridge / NUMA node; across sockets
it crosses the inter-socket link.  For the 8-GPU layout of SURVEY §2.3 PAR6
(one SSD per GPU) this module ranks every NVMe controller by that distance
from each GPU, from sysfs:

    /sys/bus/pci/devices/<bdf> -> /sys/devices/pci<dom>:<bus>/<rp>/<sw>/.../<bdf>

The chain of PCI functions on that path is the device's ancestry; two
devices' common prefix says how far up the tree their traffic must climb.
``sysfs`` is a parameter so the CPU tests run against a fake tree.

``python -m nvme_strom_amd.utils.topology [--file PATH] [--sysfs /sys]``
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import re
import sys
from typing import Dict, List, Optional

_BDF = re.compile(r"^[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]$")
_ROOT = re.compile(r"^pci[0-9a-f]{4}:[0-9a-f]{2}$")

# closer is better; used to rank controllers for a GPU
AFFINITY = ["same-switch", "same-root-port", "same-host-bridge", "same-numa", "cross-numa",
            "unknown"]


def pci_chain(bdf: str, sysfs: str = "/sys") -> List[str]:
    """[host bridge, root port, ..., bdf] for a PCI function, [] if unknown."""
    p = os.path.join(sysfs, "bus", "pci", "devices", bdf)
    try:
        real = os.path.realpath(p)
    except OSError:
        return []
    if not os.path.exists(real):
        return []
    out = []
    for comp in real.split("/"):
        if _ROOT.match(comp):
            out = [comp]
        elif _BDF.match(comp) and out:
            out.append(comp)
    return out if out and out[-1] == bdf else []


def numa_node(bdf: str, sysfs: str = "/sys") -> int:
    try:
        with open(os.path.join(sysfs, "bus", "pci", "devices", bdf, "numa_node")) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def affinity(gpu_bdf: str, ssd_bdf: str, sysfs: str = "/sys") -> str:
    g, s = pci_chain(gpu_bdf, sysfs), pci_chain(ssd_bdf, sysfs)
    if not g or not s:
        return "unknown"
    if g[0] == s[0]:
        common = 0
        for a, b in zip(g[1:-1], s[1:-1]):   # shared bridges above both devices
            if a != b:
                break
            common += 1
        if common >= 2:
            return "same-switch"             # a switch port below a shared root port
        if common == 1:
            return "same-root-port"
        return "same-host-bridge"
    ng, ns = numa_node(gpu_bdf, sysfs), numa_node(ssd_bdf, sysfs)
    if ng >= 0 and ng == ns:
        return "same-numa"
    return "cross-numa" if ng >= 0 and ns >= 0 else "unknown"


def nvme_controllers(sysfs: str = "/sys") -> Dict[str, str]:
    """{controller name: PCI function} from /sys/class/nvme."""
    out = {}
    base = os.path.join(sysfs, "class", "nvme")
    try:
        names = sorted(os.listdir(base))
    except OSError:
        return out
    for n in names:
        real = os.path.realpath(os.path.join(base, n, "device"))
        bdf = os.path.basename(real)
        if _BDF.match(bdf):
            out[n] = bdf
    return out


def amd_gpus(sysfs: str = "/sys") -> List[str]:
    """PCI functions of AMD GPUs (vendor 0x1002, display / accelerator class)."""
    out = []
    base = os.path.join(sysfs, "bus", "pci", "devices")
    try:
        names = sorted(os.listdir(base))
    except OSError:
        return out
    for bdf in names:
        try:
            with open(os.path.join(base, bdf, "vendor")) as f:
                vendor = f.read().strip()
            with open(os.path.join(base, bdf, "class")) as f:
                cls = int(f.read().strip(), 16)
        except (OSError, ValueError):
            continue
        if vendor == "0x1002" and (cls >> 16) in (0x03, 0x12):
            out.append(bdf)
    return out


def rank_controllers(gpu_bdf: str, sysfs: str = "/sys") -> List[dict]:
    """NVMe controllers ordered nearest-first for one GPU."""
    rows = [dict(ctrl=n, pci=b, affinity=affinity(gpu_bdf, b, sysfs),
                 numa=numa_node(b, sysfs)) for n, b in nvme_controllers(sysfs).items()]
    rows.sort(key=lambda r: (AFFINITY.index(r["affinity"]), r["ctrl"]))
    return rows


def gpu_bdf(device: int) -> Optional[str]:
    from .. import _native as N
    lib = N.lib()
    if not N.has("strom_gpu_pci_bdf"):
        return None
    buf = C.create_string_buffer(32)
    return buf.value.decode() if lib.strom_gpu_pci_bdf(device, buf, 32) == 0 else None


class _FileTopo(C.Structure):
    _fields_ = [("dev_major", C.c_uint32), ("dev_minor", C.c_uint32), ("numa_node", C.c_int32),
                ("nmembers", C.c_uint32), ("fs_name", C.c_char * 16), ("disk", C.c_char * 32),
                ("member_disk", (C.c_char * 32) * 16), ("member_pci", (C.c_char * 16) * 16)]


def file_topology(path: str) -> dict:
    """Backing disk, members and controller PCI functions of a file (native
    classification, the same CHECK_FILE uses)."""
    from .. import _native as N
    from ..api import _check
    fd = os.open(path, os.O_RDONLY)
    try:
        t = _FileTopo()
        _check(N.lib().strom_file_topology(fd, C.byref(t)), "file_topology")
    finally:
        os.close(fd)
    members = [dict(disk=t.member_disk[i].value.decode(), pci=t.member_pci[i].value.decode())
               for i in range(t.nmembers)]
    return dict(dev=f"{t.dev_major}:{t.dev_minor}", fs=t.fs_name.decode(), disk=t.disk.decode(),
                numa_node=t.numa_node, members=members)


def file_affinity(path: str, device: Optional[int] = None, sysfs: str = "/sys") -> dict:
    """File topology plus each member's affinity to a GPU (current device by
    default); the worst member bounds a striped read."""
    topo = file_topology(path)
    g = None
    if device is not None:
        g = gpu_bdf(device)
    topo["gpu_pci"] = g
    worst = "unknown" if not topo["members"] else AFFINITY[0]
    for m in topo["members"]:
        m["affinity"] = affinity(g, m["pci"], sysfs) if g and m["pci"] else "unknown"
        if AFFINITY.index(m["affinity"]) > AFFINITY.index(worst):
            worst = m["affinity"]
    topo["affinity"] = worst if topo["members"] else "virtual-fs"
    return topo


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sysfs", default="/sys")
    ap.add_argument("--file", default="")
    ap.add_argument("--device", type=int, default=None, help="HIP device for --file affinity")
    a = ap.parse_args(argv)
    out = dict(gpus=[dict(pci=g, numa=numa_node(g, a.sysfs), nvme=rank_controllers(g, a.sysfs))
                     for g in amd_gpus(a.sysfs)],
               nvme=nvme_controllers(a.sysfs))
    if a.file:
        out["file"] = file_affinity(a.file, a.device, a.sysfs)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
