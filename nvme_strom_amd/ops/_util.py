"""Shared helpers for the HIP kernel wrappers."""
from __future__ import annotations

import torch

from .. import _native as N


def lib():
    return N.lib()


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: torch.Tensor) -> int:
    return int(t.data_ptr())


def require_cuda(t: torch.Tensor, name: str, contiguous: bool = True) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HBM) tensor")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def as_u8(t: torch.Tensor) -> torch.Tensor:
    return t.view(torch.uint8) if t.dtype != torch.uint8 else t
