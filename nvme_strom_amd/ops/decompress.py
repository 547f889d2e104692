"""GPU LZ4 / snappy decode (csrc/kernels/decompress.hip) + host codec helpers.

``decompress`` takes a device byte tensor holding many compressed streams and
a descriptor per stream (source offset/length, destination offset/capacity)
and decodes them all in one launch, one wavefront per stream.  Supported:
raw LZ4 blocks, LZ4 *frames* (linked or independent blocks — the format
pyarrow's ``lz4``/``lz4_frame`` codec and Arrow IPC buffer compression use),
raw snappy and stored copies.  Host encoders/decoders (native, in libstrom)
produce test data and serve as CPU references.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native as N
from ._util import check, lib, ptr, require_cuda, stream_handle

LZ4 = 1
SNAPPY = 2
COPY = 3
LZ4_FRAME = 4
LZ4_FRAME_BCS = 5
ARROW_LZ4 = 6          # Arrow IPC buffer: i64 length prefix (-1 = raw) + LZ4 frame
ZSTD = 7               # Zstandard frame(s), RFC 8878 (csrc/kernels/zstd.hip)
ARROW_ZSTD = 8         # Arrow IPC buffer: i64 length prefix (-1 = raw) + zstd frame

# decompress(): a stream whose compressed size is at least this share of its
# capacity goes to the lane decoder
LANES_RATIO = 0.9

DESC_DTYPE = np.dtype([("src_off", "<u8"), ("dst_off", "<u8"), ("src_len", "<u4"),
                       ("dst_len", "<u4")])


# ------------------------------------------------------------ host codecs
def _host(fn, data: bytes, cap: int) -> bytes:
    src = np.frombuffer(data, dtype=np.uint8)
    out = np.empty(max(cap, 16), dtype=np.uint8)
    n = fn(src.ctypes.data, len(src), out.ctypes.data, len(out))
    if n < 0:
        raise ValueError(f"codec error {n}")
    return out[:n].tobytes()


def lz4_compress(data: bytes) -> bytes:
    return _host(N.lib().strom_lz4_compress_host, data, len(data) + len(data) // 255 + 64)


def lz4_decompress(data: bytes, size: int) -> bytes:
    return _host(N.lib().strom_lz4_decompress_host, data, size)


def snappy_compress(data: bytes) -> bytes:
    return _host(N.lib().strom_snappy_compress_host, data, 32 + len(data) + len(data) // 6)


def snappy_decompress(data: bytes, size: int) -> bytes:
    return _host(N.lib().strom_snappy_decompress_host, data, size)


@dataclass
class Lz4FrameInfo:
    data_offset: int          # first block header, relative to the frame start
    block_checksum: bool
    content_size: int         # -1 when absent
    block_max: int


def parse_lz4_frame_header(buf: bytes, off: int = 0) -> Lz4FrameInfo:
    """Parse an LZ4 frame header (magic 0x184D2204)."""
    magic, = struct.unpack_from("<I", buf, off)
    if magic != 0x184D2204:
        raise ValueError("not an LZ4 frame")
    flg, bd = buf[off + 4], buf[off + 5]
    if (flg >> 6) != 1:
        raise ValueError("unsupported LZ4 frame version")
    p = off + 6
    csize = -1
    if flg & 0x08:
        csize, = struct.unpack_from("<Q", buf, p)
        p += 8
    if flg & 0x01:
        p += 4                # dictionary id
    p += 1                    # header checksum
    block_max = {4: 64 << 10, 5: 256 << 10, 6: 1 << 20, 7: 4 << 20}.get((bd >> 4) & 7, 4 << 20)
    return Lz4FrameInfo(p - off, bool(flg & 0x10), csize, block_max)


def lz4_frame_compress(data: bytes, block_size: int = 64 << 10, linked: bool = True) -> bytes:
    """Minimal LZ4 frame writer (tests): independent raw blocks; with
    ``linked`` the flag says linked (blocks still self-contained — valid)."""
    flg = 0x40 | (0x00 if linked else 0x20)
    bd = {64 << 10: 4, 256 << 10: 5, 1 << 20: 6, 4 << 20: 7}[block_size] << 4
    hdr = bytes([0x04, 0x22, 0x4D, 0x18, flg, bd])
    hc = (_xxh32(hdr[4:]) >> 8) & 0xFF
    out = [hdr, bytes([hc])]
    for i in range(0, len(data), block_size):
        blk = data[i:i + block_size]
        c = lz4_compress(blk)
        if len(c) >= len(blk):
            out.append(struct.pack("<I", len(blk) | 0x80000000) + blk)
        else:
            out.append(struct.pack("<I", len(c)) + c)
    out.append(b"\0\0\0\0")
    return b"".join(out)


def _xxh32(data: bytes, seed: int = 0) -> int:
    try:
        import xxhash
        return xxhash.xxh32_intdigest(data, seed)
    except Exception:  # header checksum is not checked by our decoder
        return 0


_HOST = {}


def lz4par_host(codec: int, data: bytes, cap: int, threads=256):
    """The block-parallel decoder's phases (csrc/kernels/lz4par.hip) run on
    the CPU, thread by thread: -> (status, output bytes, stats dict).  The
    reference for the GPU kernel's algorithm; ``threads=512`` runs the
    geometry of the 512-thread build (lz4par_nt512.hip), ``"512b"`` that of
    the 8 KiB-batch build (lz4par_nt512_ob8k.hip)."""
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    st = np.zeros(8, dtype=np.uint32)
    if threads in (512, "512b"):
        if threads not in _HOST:
            import os
            name = "libstrom_lz4par512_host.so" if threads == 512 else "libstrom_lz4par512b_host.so"
            lib = C.CDLL(os.path.join(os.path.dirname(N.LIB_PATH), name))
            lib.strom_lz4par_host.restype = C.c_int
            lib.strom_lz4par_host.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p,
                                              C.c_uint32, C.c_void_p]
            _HOST[threads] = lib.strom_lz4par_host
        fn = _HOST[threads]
    elif threads == 256:
        fn = N.lib().strom_lz4par_host
    else:
        raise ValueError("threads: 256, 512 or '512b'")
    n = fn(codec, src.ctypes.data, len(data), out.ctypes.data, cap, st.ctypes.data)
    stats = dict(windows=int(st[0]), rounds=int(st[1]), fixes=int(st[2]), doubling=int(st[3]),
                 serial_windows=int(st[4]), serial_steps=int(st[5]), walk_windows=int(st[6]))
    return n, (out[:n].tobytes() if n >= 0 else b""), stats


ZSTD_LP = 2      # zstd_mode: the lane-parallel decoder (zstd.hip "lane-parallel")


def zstd_host_lp(codec: int, bufs, caps, ent_factor: float = 0.0):
    """The lane-parallel zstd decoder's phases on the CPU over several
    streams at once (walk, entropy groups lane by lane, executions):
    -> (statuses, outputs, streams the LP path took)."""
    n = len(bufs)
    src = np.frombuffer(b"".join(bufs) + b"\0", dtype=np.uint8)
    d = np.zeros(n, dtype=DESC_DTYPE)
    so = np.cumsum([0] + [len(b) for b in bufs])[:-1]
    do = np.cumsum([0] + list(caps))[:-1]
    d[DESC_DTYPE.names[0]], d[DESC_DTYPE.names[1]] = so, do
    d[DESC_DTYPE.names[2]], d[DESC_DTYPE.names[3]] = [len(b) for b in bufs], caps
    out = np.zeros(max(int(sum(caps)), 1), dtype=np.uint8)
    st = np.zeros(n, dtype=np.int32)
    taken = N.lib().strom_zstd_host_lp(codec, src.ctypes.data, d.ctypes.data, n, out.ctypes.data,
                                       st.ctypes.data, float(ent_factor))
    outs = [out[o:o + s].tobytes() if s >= 0 else b"" for o, s in zip(do, st.tolist())]
    return st.tolist(), outs, taken


def zstd_host(codec: int, data: bytes, cap: int, fp: int = 0, lp: bool = False):
    """The zstd kernel's phases run lane by lane on the CPU
    (csrc/kernels/zstd.hip): -> (status, output bytes).  The reference for
    the GPU decoder; status = decoded bytes or <0 (-1 malformed,
    -2 overflow, -3 distance, -4 unsupported: a dictionary).  ``fp`` = 2..8
    runs the frame-parallel decoder's phases (that many blocks per group,
    waves one after another)."""
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    if lp:
        st, outs, _ = zstd_host_lp(codec, [bytes(data)], [cap])
        return st[0], outs[0]
    if fp:
        n = N.lib().strom_zstd_host_fp(codec, src.ctypes.data, len(data), out.ctypes.data, cap, fp)
    else:
        n = N.lib().strom_zstd_host(codec, src.ctypes.data, len(data), out.ctypes.data, cap)
    return n, (out[:n].tobytes() if n >= 0 else b"")


def arrow_zstd_buffer(data: bytes, frame: bytes) -> bytes:
    """An Arrow IPC compressed buffer: i64 uncompressed length + zstd frame."""
    return struct.pack("<q", len(data)) + frame


def arrow_lz4_buffer(data: bytes, frame: bytes) -> bytes:
    """An Arrow IPC compressed buffer: i64 uncompressed length + LZ4 frame."""
    return struct.pack("<q", len(data)) + frame


# ------------------------------------------------------------ GPU decode
def make_descs(items: Sequence[tuple]) -> np.ndarray:
    """items: (src_off, src_len, dst_off, dst_len) per stream."""
    if len(items) == 0:
        return np.zeros(0, dtype=DESC_DTYPE)
    a = np.asarray(items, dtype=np.int64).reshape(-1, 4)
    return make_descs_arrays(a[:, 0], a[:, 1], a[:, 2], a[:, 3])


def make_descs_arrays(src_off, src_len, dst_off, dst_len) -> np.ndarray:
    """The same from four equal-length integer arrays (no per-stream Python)."""
    d = np.zeros(len(src_off), dtype=DESC_DTYPE)
    d[DESC_DTYPE.names[0]] = src_off
    d[DESC_DTYPE.names[1]] = dst_off
    d[DESC_DTYPE.names[2]] = src_len
    d[DESC_DTYPE.names[3]] = dst_len
    return d


def decompress_async(codec: int, src: torch.Tensor, dst: torch.Tensor, d_desc: torch.Tensor,
                     status: torch.Tensor, stream=None, lanes: bool = False,
                     zstd_mode: Optional[int] = None) -> None:
    """Device-side descriptors (uint8 view of DESC_DTYPE records) and status:
    no host sync; the caller checks ``status`` on the device.  Bounds are
    the caller's contract (checked by :func:`decompress`).  ``lanes``: the
    lane-group LZ4 decoder whatever the stream count — the faster one for
    literal-heavy streams (a serial parse with few tokens, wide literal
    copies; profiles/r4/dec/lz4par_chars.json).  ``zstd_mode``: the zstd
    decoder for this launch (0 one wave per stream, 1 frame-parallel,
    2 lane-parallel, None / -1 the library's choice)."""
    n = d_desc.numel() // DESC_DTYPE.itemsize
    if n == 0:
        return
    if zstd_mode == ZSTD_LP and codec in (ZSTD, ARROW_ZSTD):
        # the entry pool is sized from the decoded capacity (dst)
        check(lib().strom_decompress_zstd_lp(codec, ptr(src), ptr(dst), ptr(d_desc), n,
                                             ptr(status), dst.numel(), stream_handle(stream)),
              "decompress")
        return
    if zstd_mode is not None and codec in (ZSTD, ARROW_ZSTD):
        check(lib().strom_decompress_zstd_mode(codec, ptr(src), ptr(dst), ptr(d_desc), n,
                                               ptr(status), None, 0, stream_handle(stream),
                                               int(zstd_mode)), "decompress")
        return
    fn = lib().strom_decompress_lanes if lanes else lib().strom_decompress
    check(fn(codec, ptr(src), ptr(dst), ptr(d_desc), n, ptr(status), stream_handle(stream)),
          "decompress")


def decompress(codec: int, src: torch.Tensor, dst: torch.Tensor, descs: np.ndarray,
               stream=None) -> np.ndarray:
    """Decode every stream described by ``descs``; returns per-stream status
    (decoded byte count, or <0: -1 malformed, -2 overflow)."""
    require_cuda(src, "src")
    require_cuda(dst, "dst")
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    for name, t in (("src", src), ("dst", dst)):
        if t.dtype != torch.uint8:
            raise ValueError(f"{name} must be uint8")
    if len(descs) == 0:
        return np.zeros(0, dtype=np.int32)
    if int((descs["src_off"] + descs["src_len"]).max()) > src.numel():
        raise ValueError("descriptor source out of range")
    if int((descs["dst_off"] + descs["dst_len"]).max()) > dst.numel():
        raise ValueError("descriptor destination out of range")
    # streams stored at >= LANES_RATIO of their capacity (literal runs, a
    # token per few hundred bytes) take the lane decoder, the rest the
    # library's choice — the Arrow scan's per-buffer routing
    # (models/arrow_scan.py; profiles/r4/dec/lz4par_final.json chars, 2,048
    # streams: LZ4 lanes 173 vs block-parallel 108 GB/s, snappy 402 vs 316).
    # A decoder forced with STROM_DECOMP_PAR takes every stream.
    if codec in (LZ4, LZ4_FRAME, LZ4_FRAME_BCS, ARROW_LZ4, SNAPPY) and \
            os.environ.get("STROM_DECOMP_PAR") is None:
        lit = descs["src_len"].astype(np.float64) >= LANES_RATIO * descs["dst_len"]
    else:
        lit = np.zeros(len(descs), dtype=bool)
    status = torch.empty(len(descs), dtype=torch.int32, device=src.device)
    for mask, fn in ((~lit, lib().strom_decompress), (lit, lib().strom_decompress_lanes)):
        idx = np.nonzero(mask)[0]
        if not len(idx):
            continue
        part = descs if len(idx) == len(descs) else descs[idx]
        d_desc = torch.from_numpy(part.view(np.uint8).copy()).to(src.device)
        st = status if len(idx) == len(descs) else \
            torch.empty(len(idx), dtype=torch.int32, device=src.device)
        check(fn(codec, ptr(src), ptr(dst), ptr(d_desc), len(idx), ptr(st),
                 stream_handle(stream)), "decompress")
        if st is not status:
            status[torch.from_numpy(idx).to(src.device)] = st
    return status.cpu().numpy()
