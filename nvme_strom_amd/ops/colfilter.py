"""Columnar range filter + selection compaction (csrc/kernels/colfilter.hip)."""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ._util import check, lib, ptr, require_cuda, stream_handle

_TYPES = {torch.int32: 1, torch.int64: 2, torch.float32: 3, torch.float64: 4}


def column_filter(values: torch.Tensor, lo, hi, valid: Optional[torch.Tensor] = None,
                  stream=None) -> Tuple[torch.Tensor, int]:
    """Selection bitmap (int64 words, LSB-first like Arrow validity) of
    ``lo <= v <= hi`` AND valid, plus the selected count."""
    require_cuda(values, "values")
    if values.dtype not in _TYPES:
        raise ValueError(f"unsupported dtype {values.dtype}")
    n = values.numel()
    words = (n + 63) // 64
    bm = torch.empty(max(words, 1), dtype=torch.int64, device=values.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=values.device)
    vptr = 0
    if valid is not None:
        require_cuda(valid, "valid")
        if valid.numel() * valid.element_size() < words * 8:
            # Arrow pads validity to 64 bytes; pad here when a caller did not
            pad = torch.zeros(words * 8, dtype=torch.uint8, device=values.device)
            vb = valid.view(torch.uint8)
            pad[:vb.numel()] = vb
            valid = pad
        vptr = ptr(valid)
    check(lib().strom_column_filter(_TYPES[values.dtype], ptr(values), vptr, n, float(lo),
                                    float(hi), ptr(bm), ptr(cnt), stream_handle(stream)),
          "column_filter")
    return bm, int(cnt.item())


def bitmap_to_indices(bitmap: torch.Tensor, n: int, count: Optional[int] = None,
                      stream=None) -> torch.Tensor:
    """Ordered int32 row indices of the set bits (first ``n`` rows)."""
    require_cuda(bitmap, "bitmap")
    if count is None:
        count = int(_popcount(bitmap, n))
    out = torch.empty(max(count, 1), dtype=torch.int32, device=bitmap.device)
    total = torch.zeros(1, dtype=torch.int64, device=bitmap.device)
    check(lib().strom_bitmap_to_indices(ptr(bitmap), n, ptr(out), ptr(total),
                                        stream_handle(stream)), "bitmap_to_indices")
    return out[:count]


def _popcount(bitmap: torch.Tensor, n: int) -> int:
    b = bitmap.cpu().numpy().view(np.uint8)
    bits = np.unpackbits(b, bitorder="little")[:n]
    return int(bits.sum())


# ----------------------------------------------------------- batched scan
# struct strom_filter_batch (strom.h): values, valid, nrows, word_base,
# row_base as five u64 — a (nbatches, 5) int64 tensor on the device
BATCH_FIELDS = 5


def filter_batched(dtype: torch.dtype, batches: torch.Tensor, nwords: int, lo, hi,
                   bitmap: torch.Tensor, count: torch.Tensor, stream=None,
                   combine: bool = False) -> None:
    """One launch over many record batches; ``count`` (int64[1] on the
    device) accumulates the selected rows — nothing is read back.
    ``combine`` ANDs the predicate into the bitmap already there (the next
    qualifier of a conjunction; ``count`` then counts the combined rows)."""
    if dtype not in _TYPES:
        raise ValueError(f"unsupported dtype {dtype}")
    require_cuda(batches, "batches")
    nb = batches.shape[0]
    if batches.dtype != torch.int64 or batches.shape[1] != BATCH_FIELDS:
        raise ValueError("batches: int64 (n, 5)")
    if bitmap.numel() < nwords:
        raise ValueError("bitmap too small")
    check(lib().strom_column_filter_batched2(_TYPES[dtype], ptr(batches), nb, nwords, float(lo),
                                             float(hi), ptr(bitmap), ptr(count), int(combine),
                                             stream_handle(stream)), "column_filter_batched")


def bitmap_to_rows(bitmap: torch.Tensor, nwords: int, batches: torch.Tensor, out: torch.Tensor,
                   cursor: torch.Tensor, stream=None, proj: Optional[torch.Tensor] = None,
                   proj_out: Optional[torch.Tensor] = None,
                   proj_valid: Optional[torch.Tensor] = None) -> None:
    """Append global row ids (int64) of the set bits at ``out[cursor]``;
    ``cursor`` (int64[1], device) advances — successive groups of one scan
    fill ``out`` in order without a host round trip.  ``proj`` (a batch
    table of another column, same batches) gathers that column's value of
    each selected row into ``proj_out[cursor]`` (1/2/4/8-byte elements),
    and its validity (0/1) into ``proj_valid`` when given."""
    require_cuda(bitmap, "bitmap")
    if out.dtype != torch.int64:
        raise ValueError("out must be int64")
    width, pptr, vptr = 0, 0, 0
    if proj is not None:
        if proj_out is None or proj.shape != batches.shape:
            raise ValueError("projection needs proj_out and a table of the same batches")
        width = proj_out.element_size() * (proj_out.shape[1] if proj_out.dim() == 2 else 1)
        if width not in (1, 2, 4, 8, 16):
            raise ValueError("projected values are 1, 2, 4, 8 or 16 bytes")
        pptr = ptr(proj_out)
        vptr = ptr(proj_valid) if proj_valid is not None else 0
    check(lib().strom_bitmap_to_rows_proj(ptr(bitmap), nwords, ptr(batches), batches.shape[0],
                                          ptr(out), ptr(cursor),
                                          ptr(proj) if proj is not None else 0, width, pptr,
                                          vptr, stream_handle(stream)), "bitmap_to_rows")


def bitmap_to_rows_str(bitmap: torch.Tensor, nwords: int, batches: torch.Tensor, out: torch.Tensor,
                       cursor: torch.Tensor, strtab: torch.Tensor, owidth: int,
                       poff: torch.Tensor, pchars: torch.Tensor, char_cursor: torch.Tensor,
                       pvalid: Optional[torch.Tensor] = None, stream=None) -> None:
    """bitmap_to_rows with a utf8/binary column projected: ``strtab`` is its
    (nbatches, 7) strom_qual_batch table (offsets of ``owidth`` bytes, the
    characters in aux); each selected row's characters are appended at the
    device cursor ``char_cursor`` in ``pchars`` and their start written to
    ``poff`` at the row's output position."""
    require_cuda(bitmap, "bitmap")
    if out.dtype != torch.int64 or poff.dtype != torch.int64 or pchars.dtype != torch.uint8:
        raise ValueError("out / poff int64, pchars uint8")
    if strtab.shape[0] != batches.shape[0] or strtab.shape[1] != 7:
        raise ValueError("strtab: (nbatches, 7) of the same batches")
    check(lib().strom_bitmap_to_rows_str(ptr(bitmap), nwords, ptr(batches), batches.shape[0],
                                         ptr(out), ptr(cursor), ptr(strtab), owidth, ptr(poff),
                                         ptr(pchars), ptr(pvalid) if pvalid is not None else 0,
                                         ptr(char_cursor), stream_handle(stream)),
          "bitmap_to_rows_str")
