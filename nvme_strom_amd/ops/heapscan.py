"""PostgreSQL heap-page scan on the GPU (csrc/kernels/heapscan.hip)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .. import _native as N
from ._util import check, lib, ptr, require_cuda, stream_handle

VERIFY_CHECKSUM = 1
SKIP_INVISIBLE = 2
PAGE_BAD_HEADER = 1
PAGE_BAD_CHECKSUM = 2
PAGE_EMPTY = 4


@dataclass
class HeapScanResult:
    items: torch.Tensor        # int32 (page << 16 | lineno), unordered
    count: int
    page_status: torch.Tensor  # int32 per page (PAGE_* bits)

    def sorted_items(self) -> np.ndarray:
        return np.sort(self.items[:self.count].cpu().numpy().view(np.uint32))


def heap_scan(pages: torch.Tensor, page_sz: int = 8192, verify_checksum: bool = False,
              skip_invisible: bool = False, attr_off: int = -1, attr_width: int = 4,
              lo: int = -(1 << 63), hi: int = (1 << 63) - 1, blkno_base: int = 0,
              out_cap: Optional[int] = None, blknos: Optional[torch.Tensor] = None,
              stream=None) -> HeapScanResult:
    """Scan ``pages`` (uint8, npages*page_sz) for visible LP_NORMAL tuples,
    optionally filtered by lo <= int column at ``attr_off`` (after t_hoff) <= hi."""
    require_cuda(pages, "pages")
    pages = pages.view(torch.uint8)
    if pages.numel() % page_sz:
        raise ValueError("pages is not a whole number of pages")
    npages = pages.numel() // page_sz
    cap = out_cap if out_cap is not None else npages * (page_sz // 28 + 1)
    items = torch.empty(max(cap, 1), dtype=torch.int32, device=pages.device)
    count = torch.zeros(1, dtype=torch.int32, device=pages.device)
    status = torch.empty(max(npages, 1), dtype=torch.int32, device=pages.device)
    flags = (VERIFY_CHECKSUM if verify_checksum else 0) | (SKIP_INVISIBLE if skip_invisible else 0)
    a = N.HeapScanArgs(pages=ptr(pages), npages=npages, page_sz=page_sz, flags=flags,
                       attr_off=attr_off, attr_width=attr_width, lo=lo, hi=hi,
                       out_items=ptr(items), out_cap=cap, out_count=ptr(count),
                       page_status=ptr(status), blkno_base=blkno_base,
                       blknos=ptr(blknos) if blknos is not None else None)
    check(lib().strom_heap_scan(C.byref(a), stream_handle(stream)), "heap_scan")
    n = int(count.item())
    return HeapScanResult(items, min(n, cap), status[:npages])
