"""Chunk reorder kernels (csrc/kernels/copyops.hip).

MEMCPY_SSD2GPU lands storage chunks packed from the head of the destination
and page-cache chunks at the tail, and rewrites ``chunk_ids`` to that landing
order (reference kmod/nvme_strom.c:1546-1571).  ``landing_positions`` turns
(requested order, landing order) into the scatter map and ``chunk_scatter``
restores the requested order on the GPU in one pass.
"""
from __future__ import annotations

from collections import defaultdict, deque

import numpy as np
import torch

from ._util import as_u8, check, lib, ptr, require_cuda, stream_handle


def landing_positions(requested: np.ndarray, landed: np.ndarray, nr_ssd: int) -> np.ndarray:
    """pos[i] = index in ``requested`` of the chunk that landed at slot i.

    Storage chunks keep their relative order; page-cache chunks fill the tail
    backwards, so the tail is matched from its end.  Duplicated ids are
    matched first-come-first-served."""
    requested = np.asarray(requested, dtype=np.uint32)
    landed = np.asarray(landed, dtype=np.uint32)
    n = len(requested)
    if nr_ssd == n and np.array_equal(requested, landed):
        return np.arange(n, dtype=np.uint32)
    where = defaultdict(deque)
    for j, c in enumerate(requested.tolist()):
        where[c].append(j)
    pos = np.empty(n, dtype=np.uint32)
    order = list(range(nr_ssd)) + list(range(n - 1, nr_ssd - 1, -1))
    for i in order:
        pos[i] = where[int(landed[i])].popleft()
    return pos


def chunk_scatter(src: torch.Tensor, dst: torch.Tensor, pos, chunk: int, stream=None) -> None:
    """dst[pos[i]*chunk : +chunk] = src[i*chunk : +chunk] for every landed chunk i."""
    src, dst = as_u8(src), as_u8(dst)
    if not src.is_cuda and not dst.is_cuda:
        # host-emulated HBM (CPU tests): same semantics, plain torch indexing
        p = torch.as_tensor(np.asarray(pos, dtype=np.int64))
        dst.view(-1, chunk)[p] = src[:len(p) * chunk].view(-1, chunk)
        return
    require_cuda(src, "src")
    require_cuda(dst, "dst")
    if not isinstance(pos, torch.Tensor):
        pos = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.uint32).view(np.int32))
    pos = pos.to(src.device, non_blocking=True)
    n = pos.numel()
    if n * chunk > src.numel() or int(pos.max().item() + 1) * chunk > dst.numel():
        raise ValueError("scatter out of range")
    check(lib().strom_chunk_scatter(ptr(src), ptr(dst), ptr(pos), n, chunk,
                                    stream_handle(stream)), "chunk_scatter")


def chunk_gather(src: torch.Tensor, dst: torch.Tensor, idx, chunk: int, stream=None) -> None:
    """dst[i*chunk : +chunk] = src[idx[i]*chunk : +chunk]."""
    src, dst = as_u8(src), as_u8(dst)
    require_cuda(src, "src")
    require_cuda(dst, "dst")
    if not isinstance(idx, torch.Tensor):
        idx = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.uint32).view(np.int32))
    idx = idx.to(src.device, non_blocking=True)
    n = idx.numel()
    if n * chunk > dst.numel() or int(idx.max().item() + 1) * chunk > src.numel():
        raise ValueError("gather out of range")
    check(lib().strom_chunk_gather(ptr(src), ptr(dst), ptr(idx), n, chunk,
                                   stream_handle(stream)), "chunk_gather")
