"""On-GPU integrity checks (csrc/kernels/crc32c.hip, copyops.hip).

The reference verifies a loaded segment by copying it back to the host and
memcmp'ing against pread (utils/nvme_test.c:226-267).  Here the check stays
on the device: CRC32C per chunk (or folded over the buffer) compared with
the host CRC of the file, or a pattern / buffer comparison that returns the
mismatch count and first offset.
"""
from __future__ import annotations

import numpy as np
import torch

from ._util import as_u8, check, lib, ptr, require_cuda, stream_handle


def crc32c_chunks(buf: torch.Tensor, chunk: int, nbytes: int | None = None,
                  out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Per-chunk CRC32C of a device buffer -> int32 tensor (bit pattern = u32)."""
    buf = as_u8(buf)
    require_cuda(buf, "buf")
    n = buf.numel() if nbytes is None else int(nbytes)
    nch = (n + chunk - 1) // chunk
    if out is None:
        out = torch.empty(nch, dtype=torch.int32, device=buf.device)
    check(lib().strom_crc32c_chunks(ptr(buf), n, chunk, ptr(out), stream_handle(stream)),
          "crc32c_chunks")
    return out


def crc32c(buf: torch.Tensor, nbytes: int | None = None, chunk: int = 1 << 16,
           stream=None) -> int:
    """CRC32C of the whole buffer (per-chunk kernel + GF(2) fold kernel)."""
    buf = as_u8(buf)
    n = buf.numel() if nbytes is None else int(nbytes)
    if n == 0:
        return 0
    per = crc32c_chunks(buf, chunk, n, stream=stream)
    out = torch.empty(1, dtype=torch.int32, device=buf.device)
    check(lib().strom_crc32c_combine(ptr(per), per.numel(), chunk, n, ptr(out),
                                     stream_handle(stream)), "crc32c_combine")
    return int(out.cpu().numpy().view(np.uint32)[0])


def crc32c_into(buf: torch.Tensor, out: torch.Tensor, chunk: int = 1 << 16,
                stream=None) -> None:
    """CRC32C of the whole buffer written to ``out`` (a one-element device
    int32 tensor, u32 bit pattern) on ``stream``: no host read, for checks
    that stay on the device (parallel/fanout.py's per-step slice check)."""
    buf = as_u8(buf)
    n = buf.numel()
    if n == 0:
        out.zero_()
        return
    per = crc32c_chunks(buf, chunk, n, stream=stream)
    check(lib().strom_crc32c_combine(ptr(per), per.numel(), chunk, n, ptr(out),
                                     stream_handle(stream)), "crc32c_combine")


def u32(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy().view(np.uint32)


def verify_pattern(buf: torch.Tensor, pattern: int, stream=None) -> tuple[int, int]:
    """-> (mismatching 4-byte words, first mismatching byte offset or -1)."""
    buf = as_u8(buf)
    require_cuda(buf, "buf")
    out = torch.empty(2, dtype=torch.int64, device=buf.device)
    check(lib().strom_verify_pattern(ptr(buf), buf.numel(), pattern & 0xffffffff, ptr(out),
                                     stream_handle(stream)), "verify_pattern")
    bad, first = out.cpu().numpy().view(np.uint64)
    return int(bad), (-1 if first == np.uint64(0xFFFFFFFFFFFFFFFF) else int(first))


def verify_equal(a: torch.Tensor, b: torch.Tensor, stream=None) -> tuple[int, int]:
    a, b = as_u8(a), as_u8(b)
    require_cuda(a, "a")
    require_cuda(b, "b")
    if a.numel() != b.numel():
        raise ValueError("size mismatch")
    out = torch.empty(2, dtype=torch.int64, device=a.device)
    check(lib().strom_verify_equal(ptr(a), ptr(b), a.numel(), ptr(out), stream_handle(stream)),
          "verify_equal")
    bad, first = out.cpu().numpy().view(np.uint64)
    return int(bad), (-1 if first == np.uint64(0xFFFFFFFFFFFFFFFF) else int(first))


def fill_pattern(buf: torch.Tensor, pattern: int, stream=None) -> None:
    buf = as_u8(buf)
    require_cuda(buf, "buf")
    check(lib().strom_fill_pattern(ptr(buf), buf.numel(), pattern & 0xffffffff,
                                   stream_handle(stream)), "fill_pattern")
