"""NUMA helpers (reference pgsql/nvme_strom.c:300-393 bind/unbind,
utils/ssd2ram_test.c:66-119 setup_cpu_affinity).

``bind_to_node`` restricts the calling process to the CPUs of a node
(intersected with what the cgroup allows) and remembers the previous mask so
``unbind`` restores it — the reference's unbind set *all* CPUs instead.
``gpu_numa_node`` reads the node of a GPU's PCIe root from sysfs.
"""
from __future__ import annotations

import os
from typing import List, Optional, Set

_saved: Optional[Set[int]] = None


def parse_cpulist(text: str) -> List[int]:
    cpus: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def node_cpus(node: int) -> List[int]:
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return parse_cpulist(f.read())
    except OSError:
        return []


def nodes() -> List[int]:
    try:
        return sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node")
                      if d.startswith("node") and d[4:].isdigit())
    except OSError:
        return []


def bind_to_node(node: int) -> bool:
    global _saved
    want = set(node_cpus(node))
    allowed = os.sched_getaffinity(0)
    use = want & allowed
    if not use:
        return False
    if _saved is None:
        _saved = set(allowed)
    os.sched_setaffinity(0, use)
    return True


def unbind() -> None:
    global _saved
    if _saved is not None:
        os.sched_setaffinity(0, _saved)
        _saved = None


def gpu_numa_node(device_index: int = 0) -> int:
    """NUMA node of a GPU's PCIe root (-1 if unknown)."""
    try:
        import torch
        props = torch.cuda.get_device_properties(device_index)
        bus = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            return int(f.read().strip())
    except Exception:
        return -1
