"""Pythonic surface over the ioctl ABI.

One call per reference ioctl (kmod/nvme_strom.h:17-28): ``check_file``,
``map_gpu_memory`` / ``unmap_gpu_memory`` / ``list_gpu_memory`` /
``info_gpu_memory``, ``alloc_dma_buffer``, ``memcpy_ssd2gpu``,
``memcpy_ssd2ram``, ``memcpy_wait`` and ``stat_info``, plus the MI355X
additions (timed wait, latency histograms, dma-buf mapping).  Errors come
back as :class:`StromError` carrying the errno and, for WAIT, the device
status of the failed task.
"""
from __future__ import annotations

import ctypes as C
import errno as _errno
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _native as N


class StromError(OSError):
    def __init__(self, err: int, what: str, status: int = 0):
        super().__init__(err, f"{what}: {os.strerror(err)}" + (f" (status {status})" if status else ""))
        self.status = status


def _check(rc: int, what: str, status: int = 0) -> int:
    if rc < 0:
        raise StromError(-rc, what, status)
    return rc


# ----------------------------------------------------------------- sessions
class Session:
    """Equivalent of one open file descriptor on /proc/nvme-strom.

    Closing a session reclaims the records of failed tasks nobody waited
    for (reference strom_proc_release, kmod/nvme_strom.c:2064-2091).
    """

    def __init__(self):
        self.lib = N.lib()
        self.sid = _check(self.lib.strom_open(), "strom_open")
        self.closed = False

    def ioctl(self, cmd: int, arg, what: str = "ioctl") -> int:
        rc = self.lib.strom_ioctl(self.sid, cmd, C.byref(arg))
        return _check(rc, what)

    def ioctl_rc(self, cmd: int, arg) -> int:
        return self.lib.strom_ioctl(self.sid, cmd, C.byref(arg))

    def close(self) -> int:
        if self.closed:
            return 0
        self.closed = True
        return self.lib.strom_close(self.sid)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


_default: Optional[Session] = None


def session() -> Session:
    global _default
    if _default is None or _default.closed:
        _default = Session()
    return _default


# ------------------------------------------------------------- config etc.
def version() -> str:
    return N.lib().strom_version().decode()


def provider() -> str:
    return "kernel" if N.lib().strom_provider() == 1 else "userspace"


def config_set(key: str, value) -> None:
    if isinstance(value, bool):
        value = int(value)
    _check(N.lib().strom_config_set(key.encode(), str(value).encode()), f"config {key}")


def config_get(key: str) -> str:
    buf = C.create_string_buffer(64)
    _check(N.lib().strom_config_get(key.encode(), buf, 64), f"config {key}")
    return buf.value.decode()


def configure(reset: bool = True, **kv) -> None:
    """Set several engine knobs; restarts the I/O workers by default."""
    for k, v in kv.items():
        config_set(k, v)
    if reset:
        engine_reset()


def engine_reset() -> None:
    N.lib().strom_engine_reset()


def fault_inject(fail_at: int = 0, err: int = _errno.EIO, short_at: int = 0,
                 short_bytes: int = 0, delay_us: int = 0) -> None:
    N.lib().strom_fault_inject(fail_at, err, short_at, short_bytes, delay_us)


def fake_backend(seed: int = 0) -> tuple:
    """Fake namespace backend counters: (completions, out-of-order
    completions); ``seed`` != 0 reseeds the completion order (next reset)."""
    c, r = C.c_uint64(), C.c_uint64()
    N.lib().strom_fake_backend(seed, C.byref(c), C.byref(r))
    return c.value, r.value


def ingest_info(device: int = 0) -> Optional[dict]:
    """Counters of the device's HBM ingest grid (the persistent GPU kernel that
    pulls staged reads into HBM), or None when it cannot run there."""
    out = np.zeros(4, dtype=np.uint64)
    if N.lib().strom_ingest_info(device, out.ctypes.data) < 0:
        return None
    return dict(available=bool(out[0]), launches=int(out[1]), posted=int(out[2]),
                outstanding=int(out[3]))


def io_info() -> dict:
    """Worker I/O facts: workers reading into io_uring-registered staging
    (READ_FIXED), registrations refused, and the last refusal's errno."""
    out = np.zeros(3, dtype=np.uint64)
    _check(N.lib().strom_io_info(out.ctypes.data), "io_info")
    return dict(fixed_workers=int(out[0]), fixed_refused=int(out[1]), fixed_errno=int(out[2]))


IO_PROF_PHASES = ("idle", "take", "start", "submit", "reap", "bar", "post", "hdp", "finish",
                  "retire", "wait")
IO_PROF_COUNTS = ("requests", "batches", "enters", "sleeps", "descriptors")


def io_prof(reset: bool = False) -> dict:
    """Per-worker phase attribution of the I/O workers (needs
    ``configure(io_prof=1)`` before the engine starts): for every phase of
    the worker loop the summed time in ns, plus ns per completed request,
    and the submitting thread's plan / build / submit time
    (``csrc/engine/io.cc`` ProfPhase)."""
    n = 2 + len(IO_PROF_PHASES) + len(IO_PROF_COUNTS) + 4
    out = np.zeros(n, dtype=np.uint64)
    _check(N.lib().strom_io_prof(out.ctypes.data, n, 1 if reset else 0), "io_prof")
    khz = max(int(out[1]), 1)
    ns = {k: int(out[2 + i]) * 1e6 / khz for i, k in enumerate(IO_PROF_PHASES)}
    cnt = {k: int(out[2 + len(IO_PROF_PHASES) + i]) for i, k in enumerate(IO_PROF_COUNTS)}
    req = max(cnt["requests"], 1)
    c0 = 2 + len(IO_PROF_PHASES) + len(IO_PROF_COUNTS)
    caller = dict(calls=int(out[c0]), **{k: round(int(out[c0 + 1 + i]) * 1e6 / khz / req, 1)
                                         for i, k in enumerate(("plan_ns_per_req", "build_ns_per_req",
                                                                "submit_ns_per_req"))})
    return dict(workers=int(out[0]), tsc_khz=khz, ns=ns, counts=cnt, caller=caller,
                ns_per_req={k: round(v / req, 1) for k, v in ns.items()},
                busy_ns_per_req=round(sum(v for k, v in ns.items() if k != "idle") / req, 1))


HOST_COSTS = ("clock_gettime", "rdtsc", "fstat", "mincore", "syscall", "mutex", "cv_notify",
              "kcmp_file", "statx_ino")


def host_costs(fd: int, n: int = 20000) -> dict:
    """ns per call of the host primitives under the 4 KiB latency path."""
    out = np.zeros(len(HOST_COSTS), dtype=np.uint64)
    _check(N.lib().strom_host_costs(fd, out.ctypes.data, n), "host_costs")
    return {k: int(v) for k, v in zip(HOST_COSTS, out)}


ENGINE_COSTS = ("registry_get", "validate", "open_file", "completion", "registry_get_cached",
                "open_file_cached", "bar_store_4k", "lock_after_bar_store", "bar_store_4k_nt",
                "lock_after_bar_store_nt", "bar_store_4k_nt_rev", "lock_after_bar_store_nt_rev",
                "bar_store_4k_movsb", "lock_after_bar_store_movsb", "bar_store_4k_two_cores",
                "two_core_handoff")


def engine_costs(handle: int, fd: int, n: int = 20000) -> dict:
    """ns per call of the engine's own steps on the synchronous 4 KiB path."""
    out = np.zeros(len(ENGINE_COSTS), dtype=np.uint64)
    _check(N.lib().strom_engine_costs(handle, fd, out.ctypes.data, n), "engine_costs")
    return {k: int(v) for k, v in zip(ENGINE_COSTS, out)}


def resident_bytes(fd: int, offset: int = 0, length: int = 1 << 62) -> int:
    return _check(N.lib().strom_resident_bytes(fd, offset, length), "resident_bytes")


def evict_file(fd: int) -> None:
    _check(N.lib().strom_evict_file(fd), "evict_file")


def crc32c_host(data, crc: int = 0) -> int:
    buf = memoryview(data).cast("B")
    arr = (C.c_char * len(buf)).from_buffer_copy(buf) if buf.readonly else (C.c_char * len(buf)).from_buffer(buf)
    return N.lib().strom_crc32c_host(crc, arr, len(buf))


# ---------------------------------------------------------------- CHECK_FILE
@dataclass
class FileInfo:
    numa_node_id: int
    support_dma64: bool


def check_file(fd: int, sess: Optional[Session] = None) -> FileInfo:
    a = N.CheckFile(fdesc=fd)
    (sess or session()).ioctl(N.CHECK_FILE, a, "CHECK_FILE")
    return FileInfo(a.numa_node_id, bool(a.support_dma64))


# ------------------------------------------------------- GPU memory mappings
@dataclass
class GpuMapping:
    handle: int
    gpu_page_sz: int
    gpu_npages: int
    vaddress: int
    length: int
    sess: Session = field(repr=False, default=None)

    def unmap(self) -> None:
        if self.handle:
            unmap_gpu_memory(self.handle, self.sess)
            self.handle = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.unmap()


def map_gpu_memory(vaddress: int, length: int, sess: Optional[Session] = None) -> GpuMapping:
    s = sess or session()
    a = N.MapGpuMemory(vaddress=vaddress, length=length)
    s.ioctl(N.MAP_GPU_MEMORY, a, "MAP_GPU_MEMORY")
    return GpuMapping(a.handle, a.gpu_page_sz, a.gpu_npages, vaddress, length, s)


def unmap_gpu_memory(handle: int, sess: Optional[Session] = None) -> None:
    a = N.UnmapGpuMemory(handle=handle)
    (sess or session()).ioctl(N.UNMAP_GPU_MEMORY, a, "UNMAP_GPU_MEMORY")


def list_gpu_memory(sess: Optional[Session] = None) -> List[int]:
    s = sess or session()
    nrooms = 64
    while True:
        a = N.list_gpu_memory_struct(nrooms)(nrooms=nrooms)
        s.ioctl(N.LIST_GPU_MEMORY, a, "LIST_GPU_MEMORY")
        if a.nitems <= nrooms:
            return [int(a.handles[i]) for i in range(a.nitems)]
        nrooms = a.nitems


def info_gpu_memory(handle: int, sess: Optional[Session] = None) -> dict:
    s = sess or session()
    nrooms = 16
    while True:
        a = N.info_gpu_memory_struct(nrooms)(handle=handle, nrooms=nrooms)
        s.ioctl(N.INFO_GPU_MEMORY, a, "INFO_GPU_MEMORY")
        if a.nitems <= nrooms:
            break
        nrooms = a.nitems
    return dict(handle=handle, nitems=a.nitems, version=a.version, gpu_page_sz=a.gpu_page_sz,
                owner=a.owner, map_offset=a.map_offset, map_length=a.map_length,
                paddrs=[int(a.paddrs[i]) for i in range(a.nitems)])


# ------------------------------------------------------------ DMA buffers
class DmaBuffer:
    """NUMA-local host buffer usable as an SSD2RAM destination.

    ``array`` is a writable numpy uint8 view of the mapping; ``address`` is
    the mapping's VA (what MEMCPY_SSD2RAM takes as ``dest_uaddr``).  The
    mapping is made by the engine (``strom_dmabuf_mmap``), so SSD2RAM finds
    it in the registry's address index; ``array`` must not be used after
    :meth:`close`.
    """

    def __init__(self, length: int, node: int = -1, sess: Optional[Session] = None):
        a = N.AllocDMABuffer(length=length, node_id=node)
        (sess or session()).ioctl(N.ALLOC_DMA_BUFFER, a, "ALLOC_DMA_BUFFER")
        self.fd = a.dmabuf_fdesc
        self.length = os.fstat(self.fd).st_size
        self.node = node
        self._lib = N.lib()
        addr = self._lib.strom_dmabuf_mmap(self.fd, self.length)
        if not addr:
            err = C.get_errno() or _errno.EINVAL
            os.close(self.fd)
            self.fd = -1
            raise StromError(err, "strom_dmabuf_mmap")
        self.address = int(addr)
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.length).from_address(self.address))

    def close(self) -> None:
        if self.fd >= 0:
            self.array = None
            self._lib.strom_dmabuf_munmap(self.address, self.length)
            os.close(self.fd)
            self.fd = -1

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def dmabuf_gc() -> int:
    """Drop DMA buffers nothing refers to any more; returns how many remain."""
    return N.lib().strom_dmabuf_gc()


def gpu_detached() -> int:
    """Mappings detached because their allocation was freed or replaced."""
    return N.lib().strom_gpu_detached()


def alloc_dma_buffer(length: int, node: int = -1, sess: Optional[Session] = None) -> DmaBuffer:
    return DmaBuffer(length, node, sess)


# -------------------------------------------------------------- stripe sets
class StripeSet:
    """A logical file striped over member files, one per SSD (SURVEY §2.3
    PAR2 without md): stripe ``s`` of ``unit`` bytes lives in member
    ``s % n`` at offset ``(s // n) * unit``.  ``fd`` is a pseudo descriptor
    the engine accepts wherever it takes a file descriptor (CHECK_FILE,
    MEMCPY_SSD2GPU / SSD2RAM, pread_gpu, FileReader / StreamLoader).
    Requests split at stripe boundaries and run on every member at once.
    """

    def __init__(self, members, unit: int = 1 << 20, size: Optional[int] = None):
        self.unit = int(unit)
        self._own = []
        fds = []
        for m in members:
            if isinstance(m, int):
                fds.append(m)
            else:
                fd = os.open(m, os.O_RDONLY)
                self._own.append(fd)
                fds.append(fd)
        self.members = list(members)
        self.size = int(size) if size is not None else sum(os.fstat(fd).st_size for fd in fds)
        arr = (C.c_int * len(fds))(*fds)
        rc = N.lib().strom_stripe_open(arr, len(fds), self.unit, self.size)
        if rc < 0:
            for fd in self._own:
                os.close(fd)
            raise StromError(-rc, "strom_stripe_open")
        self.fd = rc

    def close(self) -> None:
        if self.fd >= 0:
            N.lib().strom_stripe_close(self.fd)
            self.fd = -1
            for fd in self._own:
                os.close(fd)
            self._own = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class RegisteredFile:
    """A file registered with the engine (io_uring's registered files): the
    descriptor (or path) is resolved once and ``fd`` is an id the engine
    accepts wherever it takes a file descriptor (pread_gpu, CHECK_FILE,
    MEMCPY_SSD2GPU / SSD2RAM, the latency probes).  Reads by id skip the
    per-read identity check of a plain descriptor (kcmp or fstat): the
    engine reads through descriptors of its own, so closing the caller's
    descriptor does not end the registration; ``close()`` does."""

    def __init__(self, f):
        own = None
        if not isinstance(f, int):
            own = fd = os.open(f, os.O_RDONLY)
        else:
            fd = f
        try:
            rc = N.lib().strom_register_file(fd)
        finally:
            if own is not None:
                os.close(own)
        if rc < 0:
            raise StromError(-rc, "strom_register_file")
        self.fd = rc

    def close(self) -> None:
        if self.fd >= 0:
            N.lib().strom_unregister_file(self.fd)
            self.fd = -1

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_striped(paths, data, unit: int = 1 << 20) -> int:
    """Write ``data`` (bytes-like) as a stripe set over ``paths``; returns
    the logical size (test and benchmark helper)."""
    mv = memoryview(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray)
                    else data.view(np.uint8).reshape(-1))
    n = len(paths)
    files = [open(p, "wb") for p in paths]
    try:
        for s, off in enumerate(range(0, len(mv), unit)):
            files[s % n].write(mv[off:off + unit])
        for f in files:
            f.flush()
            os.fsync(f.fileno())
    finally:
        for f in files:
            f.close()
    return len(mv)


# ---------------------------------------------------------------- MEMCPY_*
@dataclass
class CopyResult:
    dma_task_id: int
    nr_ram: int      # chunks served from the page cache
    nr_ssd: int      # chunks read from storage
    nr_dma_submit: int
    nr_dma_blocks: int

    @property
    def avg_request_bytes(self) -> float:
        return 512.0 * self.nr_dma_blocks / self.nr_dma_submit if self.nr_dma_submit else 0.0


def _ids_array(chunk_ids) -> np.ndarray:
    ids = np.ascontiguousarray(chunk_ids, dtype=np.uint32)
    return ids


def memcpy_ssd2gpu(handle: int, offset: int, fd: int, chunk_ids: np.ndarray, chunk_sz: int,
                   relseg_sz: int = 0, wb_buffer: int = 0,
                   sess: Optional[Session] = None) -> CopyResult:
    """Issue MEMCPY_SSD2GPU.  ``chunk_ids`` (uint32, contiguous) is rewritten
    in place to the landing order: storage chunks from the head of the
    destination, page-cache chunks (copied into ``wb_buffer``'s tail) last."""
    if not (isinstance(chunk_ids, np.ndarray) and chunk_ids.dtype == np.uint32
            and chunk_ids.flags.c_contiguous):
        raise TypeError("chunk_ids must be a contiguous numpy uint32 array (rewritten in place)")
    a = N.MemCopySsdToGpu(handle=handle, offset=offset, file_desc=fd, nr_chunks=len(chunk_ids),
                          chunk_sz=chunk_sz, relseg_sz=relseg_sz,
                          chunk_ids=chunk_ids.ctypes.data_as(C.POINTER(C.c_uint32)),
                          wb_buffer=wb_buffer or None)
    (sess or session()).ioctl(N.MEMCPY_SSD2GPU, a, "MEMCPY_SSD2GPU")
    return CopyResult(a.dma_task_id, a.nr_ram2gpu, a.nr_ssd2gpu, a.nr_dma_submit, a.nr_dma_blocks)


# strom_file_extent records (uapi.h): file_off / len in, dst_off out
EXTENT_DTYPE = np.dtype([("file_off", "<u8"), ("dst_off", "<u8"), ("len", "<u4"),
                         ("reserved", "<u4")])


@dataclass
class ExtentResult:
    dma_task_id: int
    nr_dma_submit: int
    nr_dma_blocks: int
    bytes_read: int       # storage bytes the requests read
    gap_bytes: int        # bytes_read - the extents' bytes (holes + page padding)
    dst_bytes: int        # destination span used from the offset
    dst_off: np.ndarray   # uint64 per extent: where it landed, from the offset

    @property
    def avg_request_bytes(self) -> float:
        return 512.0 * self.nr_dma_blocks / self.nr_dma_submit if self.nr_dma_submit else 0.0


def extents_array(file_off, length) -> np.ndarray:
    """strom_file_extent records of (file offset, length) pairs."""
    off = np.asarray(file_off, dtype=np.uint64).reshape(-1)
    ln = np.asarray(length, dtype=np.uint64).reshape(-1)
    if off.shape != ln.shape:
        raise ValueError("file_off and length differ in length")
    if len(ln) and int(ln.max()) > 0xFFFFFFFF:
        raise ValueError("an extent longer than 4 GiB")
    x = np.zeros(len(off), dtype=EXTENT_DTYPE)
    x["file_off"], x["len"] = off, ln.astype(np.uint32)
    return x


def memcpy_ssd2gpu_extents(handle: int, offset: int, fd: int, extents: np.ndarray,
                           gap_max: int = 64 << 10, plan_only: bool = False,
                           sess: Optional[Session] = None) -> ExtentResult:
    """Issue MEMCPY_SSD2GPU_EXTENTS (uapi.h): read the byte ranges of
    ``extents`` (EXTENT_DTYPE, sorted by file offset, disjoint; its dst_off
    column is filled in place) into the mapping at ``offset``, holes of at
    most ``gap_max`` bytes read through.  ``plan_only``: the layout without
    reading (``handle`` unused) — the destination size is ``dst_bytes``."""
    if not (isinstance(extents, np.ndarray) and extents.dtype == EXTENT_DTYPE
            and extents.flags.c_contiguous):
        raise TypeError("extents must be a contiguous EXTENT_DTYPE array (dst_off written in place)")
    a = N.MemCopySsdToGpuExtents(handle=handle, offset=offset, file_desc=fd,
                                 nr_extents=len(extents), gap_max=int(gap_max),
                                 flags=N.EXTENTS_PLAN_ONLY if plan_only else 0,
                                 extents=extents.ctypes.data if len(extents) else None)
    (sess or session()).ioctl(N.MEMCPY_SSD2GPU_EXTENTS, a, "MEMCPY_SSD2GPU_EXTENTS")
    return ExtentResult(a.dma_task_id, a.nr_dma_submit, a.nr_dma_blocks, a.bytes_read,
                        a.gap_bytes, a.dst_bytes, extents["dst_off"])


def memcpy_ssd2ram(dest_addr: int, fd: int, chunk_ids, chunk_sz: int, relseg_sz: int = 0,
                   sess: Optional[Session] = None) -> CopyResult:
    ids = _ids_array(chunk_ids)
    a = N.MemCopySsdToRam(dest_uaddr=dest_addr, file_desc=fd, nr_chunks=len(ids),
                          chunk_sz=chunk_sz, relseg_sz=relseg_sz,
                          chunk_ids=ids.ctypes.data_as(C.POINTER(C.c_uint32)))
    (sess or session()).ioctl(N.MEMCPY_SSD2RAM, a, "MEMCPY_SSD2RAM")
    return CopyResult(a.dma_task_id, a.nr_ram2ram, a.nr_ssd2ram, a.nr_dma_submit, a.nr_dma_blocks)


def pread_gpu(handle: int, offset: int, fd: int, file_off: int, length: int,
              sess: Optional[Session] = None) -> int:
    """Synchronous read of file bytes into a mapped GPU range, file order
    preserved (MEMCPY_SSD2GPU + WAIT in one native call)."""
    s = sess or session()
    return _check(s.lib.strom_pread_gpu(s.sid, handle, offset, fd, file_off, length),
                  "pread_gpu")


def pread_gpu_latency(handle: int, offset: int, fd: int, file_offs, length: int = 4096,
                      sess: Optional[Session] = None) -> np.ndarray:
    """QD1 latency probe: one synchronous pread_gpu per file offset, timed in
    the native loop (the reference's C tools' vantage point).  -> ns per read."""
    s = sess or session()
    offs = np.ascontiguousarray(file_offs, dtype=np.uint64)
    out = np.zeros(len(offs), dtype=np.uint64)
    _check(s.lib.strom_pread_gpu_lat(s.sid, handle, offset, fd, offs.ctypes.data, len(offs),
                                     length, out.ctypes.data), "pread_gpu_lat")
    return out


def ioctl_latency(handle: int, offset: int, fd: int, file_offs, length: int = 4096,
                  sess: Optional[Session] = None) -> np.ndarray:
    """QD1 probe through MEMCPY_SSD2GPU + MEMCPY_WAIT per read (the v0.6
    client's call pair), native loop.  -> ns per read."""
    s = sess or session()
    offs = np.ascontiguousarray(file_offs, dtype=np.uint64)
    out = np.zeros(len(offs), dtype=np.uint64)
    _check(s.lib.strom_ioctl_lat(s.sid, handle, offset, fd, offs.ctypes.data, len(offs),
                                 length, out.ctypes.data), "ioctl_lat")
    return out


PHASES = ("lookup", "plan", "setup", "storage", "hbm_store", "hdp_flush", "complete", "wait")


def pread_gpu_phases(handle: int, offset: int, fd: int, file_offs, length: int = 4096,
                     sess: Optional[Session] = None) -> np.ndarray:
    """Phase-stamped QD1 probe: (n, len(PHASES)) ns from each read's start to
    the end of each phase (0 where a phase was not reached; last = total)."""
    s = sess or session()
    offs = np.ascontiguousarray(file_offs, dtype=np.uint64)
    out = np.zeros((len(offs), len(PHASES)), dtype=np.uint64)
    _check(s.lib.strom_pread_gpu_phases(s.sid, handle, offset, fd, offs.ctypes.data, len(offs),
                                        length, out.ctypes.data), "pread_gpu_phases")
    return out


def phase_breakdown(stamps: np.ndarray) -> dict:
    """Median duration (us) of each phase of pread_gpu_phases() stamps: a phase
    lasts from the previous reached stamp to its own; None if never reached."""
    st = stamps.astype(np.float64)
    prev = np.zeros(len(st))
    out = {}
    for k, name in enumerate(PHASES):
        col = st[:, k]
        hit = col > 0
        out[name] = round(float(np.median((col - prev)[hit])) / 1e3, 2) if hit.any() else None
        prev = np.where(hit, col, prev)
    return out


def pread_raw_latency(fd: int, file_offs, length: int = 4096) -> np.ndarray:
    """The floor under pread_gpu: O_DIRECT pread into aligned host memory,
    ns per read (no engine, no HBM)."""
    offs = np.ascontiguousarray(file_offs, dtype=np.uint64)
    out = np.zeros(len(offs), dtype=np.uint64)
    _check(N.lib().strom_pread_raw_lat(fd, offs.ctypes.data, len(offs), length, out.ctypes.data),
           "pread_raw_lat")
    return out


def pread_pair_latency(handle: int, offset: int, fd: int, file_offs, length: int = 4096,
                       sess: Optional[Session] = None) -> tuple:
    """QD1 engine read vs the raw floor at the same moment: pairs of a raw
    O_DIRECT pread (file_offs[2i]) and a pread_gpu (file_offs[2i+1]),
    interleaved, the order flipped every pair.  -> (engine ns, raw ns) per
    pair; their pairwise difference is the engine's cost over the storage
    with the storage's drift cancelled."""
    s = sess or session()
    offs = np.ascontiguousarray(file_offs, dtype=np.uint64)
    n = len(offs) // 2
    eng = np.zeros(n, dtype=np.uint64)
    raw = np.zeros(n, dtype=np.uint64)
    _check(s.lib.strom_pread_pair_lat(s.sid, handle, offset, fd, offs.ctypes.data, n, length,
                                      eng.ctypes.data, raw.ctypes.data), "pread_pair_lat")
    return eng, raw


def raw_read_rate(fd: int, block: int, nreq: int, threads: int = 4, qd: int = 8,
                  sequential: bool = False, buffered: bool = False,
                  fixed: bool = False) -> tuple:
    """Storage ceiling for one block size with no engine in the way:
    ``threads`` io_uring rings ``qd`` deep, O_DIRECT reads into host memory
    at random aligned offsets, or ``sequential``: each ring reads its own
    disjoint run of the file in order (no cursor shared between rings);
    ``buffered`` reads through the page cache instead; ``fixed``: into
    2 MiB-page buffers registered with the ring (READ_FIXED, as the
    engine's pinned staging).  Returns (IOPS, GiB/s)."""
    iops, gibps = C.c_double(), C.c_double()
    _check(N.lib().strom_raw_read_rate(fd, block, nreq, threads, qd,
                                       int(sequential) | (2 if buffered else 0) |
                                       (4 if fixed else 0),
                                       C.byref(iops), C.byref(gibps)), "raw_read_rate")
    return iops.value, gibps.value


def raw_read_list(fd: int, offs, lens, threads: int = 4, qd: int = 8, buffered: bool = False,
                  fixed: bool = False) -> tuple:
    """The raw_read_rate rings reading exactly the requests ``(offs[i],
    lens[i])`` (4 KiB aligned), ring t taking the t-th contiguous share of
    the list: the storage's own rate for the access pattern an engine call
    produced.  Returns (IOPS, GiB/s of the bytes read)."""
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    n = np.ascontiguousarray(lens, dtype=np.uint32)
    if o.shape != n.shape or o.ndim != 1:
        raise ValueError("offs and lens must be 1-D and of one length")
    iops, gibps = C.c_double(), C.c_double()
    _check(N.lib().strom_raw_read_list(fd, o.ctypes.data, n.ctypes.data, len(o), threads, qd,
                                       (2 if buffered else 0) | (4 if fixed else 0),
                                       C.byref(iops), C.byref(gibps)), "raw_read_list")
    return iops.value, gibps.value


def memcpy_wait(task_id: int, timeout: Optional[float] = None,
                sess: Optional[Session] = None) -> None:
    """Block until the task finishes; raises StromError(EIO, status=...) on a
    device error, ETIME on timeout, ENOENT for an id that was never issued."""
    s = sess or session()
    if timeout is None:
        a = N.MemCopyWait(dma_task_id=task_id)
        rc = s.ioctl_rc(N.MEMCPY_WAIT, a)
    else:
        a = N.MemCopyWaitTimed(dma_task_id=task_id, timeout_ns=int(timeout * 1e9))
        rc = s.ioctl_rc(N.MEMCPY_WAIT_TIMED, a)
    _check(rc, f"MEMCPY_WAIT({task_id})", a.status)


# --------------------------------------------------------------- statistics
def stat_info(sess: Optional[Session] = None) -> dict:
    a = N.StatInfo(version=1)
    (sess or session()).ioctl(N.STAT_INFO, a, "STAT_INFO")
    return {name: getattr(a, name) for name, _ in N.StatInfo._fields_}


def stat_hist(reset: bool = False, sess: Optional[Session] = None) -> dict:
    a = N.StatHist(version=1, reset=int(reset))
    (sess or session()).ioctl(N.STAT_HIST, a, "STAT_HIST")
    return {k: np.array(getattr(a, k)[:], dtype=np.uint64) for k in ("io_ns", "copy_ns", "task_ns")}


def hist_percentile(hist: np.ndarray, q: float) -> float:
    """Approximate percentile (ns) of a log2 histogram (bucket k = [2^(k-1), 2^k))."""
    total = int(hist.sum())
    if total == 0:
        return float("nan")
    target = q / 100.0 * total
    run = 0
    for k, c in enumerate(hist):
        if run + int(c) >= target and c:
            lo = 0.0 if k == 0 else float(1 << (k - 1))
            hi = float(1 << k)
            frac = (target - run) / float(c)
            return lo + (hi - lo) * frac
        run += int(c)
    return float(1 << (len(hist) - 1))
