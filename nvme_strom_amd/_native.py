"""ctypes binding of libstrom (csrc/, built by ``make`` / ``nvme_strom_amd.build``).

The argument blocks below are the x86-64 layouts of ``csrc/include/strom/uapi.h``
(byte-compatible with the reference's ``kmod/nvme_strom.h:33-165``); the ABI
test (tests/test_abi.py) checks them against the C static assertions.

The library is always loaded from the package tree (``nvme_strom_amd/lib``)
and loading fails loudly when it is missing: there is no pure-Python
fallback for anything that claims to run native code.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(_LIB_DIR, "libstrom.so")

# ---------------------------------------------------------------- ioctl codes
def _IO(t: str, nr: int) -> int:
    return (ord(t) << 8) | nr


CHECK_FILE = _IO("S", 0x80)
MAP_GPU_MEMORY = _IO("S", 0x81)
UNMAP_GPU_MEMORY = _IO("S", 0x82)
LIST_GPU_MEMORY = _IO("S", 0x83)
INFO_GPU_MEMORY = _IO("S", 0x84)
ALLOC_DMA_BUFFER = _IO("S", 0x85)
MAP_GPU_DMABUF = _IO("S", 0x86)
MEMCPY_SSD2GPU = _IO("S", 0x90)
MEMCPY_SSD2RAM = _IO("S", 0x91)
MEMCPY_WAIT = _IO("S", 0x92)
MEMCPY_WAIT_TIMED = _IO("S", 0x93)
MEMCPY_SSD2GPU_EXTENTS = _IO("S", 0x94)
STAT_INFO = _IO("S", 0x99)
STAT_HIST = _IO("S", 0x9A)

GPU_BOUND_SIZE = 1 << 16
HIST_BUCKETS = 48


# ------------------------------------------------------------- arg structs
class CheckFile(C.Structure):
    _fields_ = [("fdesc", C.c_int), ("numa_node_id", C.c_int), ("support_dma64", C.c_int)]


class MapGpuMemory(C.Structure):
    _fields_ = [("handle", C.c_ulong), ("gpu_page_sz", C.c_uint32), ("gpu_npages", C.c_uint32),
                ("vaddress", C.c_uint64), ("length", C.c_size_t)]


class MapGpuDmabuf(C.Structure):
    _fields_ = [("handle", C.c_ulong), ("gpu_page_sz", C.c_uint32), ("gpu_npages", C.c_uint32),
                ("dmabuf_fd", C.c_int), ("device_id", C.c_int), ("vaddress", C.c_uint64),
                ("length", C.c_size_t), ("dmabuf_offset", C.c_uint64)]


class UnmapGpuMemory(C.Structure):
    _fields_ = [("handle", C.c_ulong)]


def list_gpu_memory_struct(nrooms: int):
    class ListGpuMemory(C.Structure):
        _fields_ = [("nrooms", C.c_uint32), ("nitems", C.c_uint32),
                    ("handles", C.c_ulong * max(1, nrooms))]
    return ListGpuMemory


def info_gpu_memory_struct(nrooms: int):
    class InfoGpuMemory(C.Structure):
        _fields_ = [("handle", C.c_ulong), ("nrooms", C.c_uint32), ("nitems", C.c_uint32),
                    ("version", C.c_uint32), ("gpu_page_sz", C.c_uint32), ("owner", C.c_uint32),
                    ("map_offset", C.c_ulong), ("map_length", C.c_ulong),
                    ("paddrs", C.c_uint64 * max(1, nrooms))]
    return InfoGpuMemory


ListGpuMemory = list_gpu_memory_struct(1)
InfoGpuMemory = info_gpu_memory_struct(1)


class MemCopySsdToGpu(C.Structure):
    _fields_ = [("dma_task_id", C.c_ulong), ("nr_ram2gpu", C.c_uint), ("nr_ssd2gpu", C.c_uint),
                ("nr_dma_submit", C.c_uint), ("nr_dma_blocks", C.c_uint), ("handle", C.c_ulong),
                ("offset", C.c_size_t), ("file_desc", C.c_int), ("nr_chunks", C.c_uint),
                ("chunk_sz", C.c_uint), ("relseg_sz", C.c_uint),
                ("chunk_ids", C.POINTER(C.c_uint32)), ("wb_buffer", C.c_void_p)]


class MemCopySsdToGpuExtents(C.Structure):
    """strom_memcpy_ssd2gpu_extents (uapi.h): exact byte-range reads."""
    _fields_ = [("dma_task_id", C.c_ulong), ("nr_dma_submit", C.c_uint),
                ("nr_dma_blocks", C.c_uint), ("bytes_read", C.c_uint64),
                ("gap_bytes", C.c_uint64), ("dst_bytes", C.c_uint64), ("handle", C.c_ulong),
                ("offset", C.c_size_t), ("file_desc", C.c_int), ("nr_extents", C.c_uint),
                ("gap_max", C.c_uint), ("flags", C.c_uint), ("extents", C.c_void_p)]


EXTENTS_PLAN_ONLY = 1


class MemCopyWait(C.Structure):
    _fields_ = [("dma_task_id", C.c_ulong), ("status", C.c_long)]


class MemCopyWaitTimed(C.Structure):
    _fields_ = [("dma_task_id", C.c_ulong), ("status", C.c_long), ("timeout_ns", C.c_uint64)]


class MemCopySsdToRam(C.Structure):
    _fields_ = [("dma_task_id", C.c_ulong), ("nr_ram2ram", C.c_uint), ("nr_ssd2ram", C.c_uint),
                ("nr_dma_submit", C.c_uint), ("nr_dma_blocks", C.c_uint),
                ("dest_uaddr", C.c_void_p), ("file_desc", C.c_int), ("nr_chunks", C.c_uint),
                ("chunk_sz", C.c_uint), ("relseg_sz", C.c_uint),
                ("chunk_ids", C.POINTER(C.c_uint32))]


class AllocDMABuffer(C.Structure):
    _fields_ = [("length", C.c_size_t), ("node_id", C.c_int), ("dmabuf_fdesc", C.c_int)]


class StatInfo(C.Structure):
    _fields_ = [("version", C.c_uint), ("has_debug", C.c_ubyte), ("tsc", C.c_uint64)] + [
        (n, C.c_uint64) for n in (
            "nr_ssd2gpu", "clk_ssd2gpu", "nr_setup_prps", "clk_setup_prps", "nr_submit_dma",
            "clk_submit_dma", "nr_wait_dtask", "clk_wait_dtask", "nr_wrong_wakeup",
            "cur_dma_count", "max_dma_count", "nr_debug1", "clk_debug1", "nr_debug2",
            "clk_debug2", "nr_debug3", "clk_debug3", "nr_debug4", "clk_debug4")]


class StatHist(C.Structure):
    _fields_ = [("version", C.c_uint), ("reset", C.c_uint),
                ("io_ns", C.c_uint64 * HIST_BUCKETS), ("copy_ns", C.c_uint64 * HIST_BUCKETS),
                ("task_ns", C.c_uint64 * HIST_BUCKETS)]


class HeapScanArgs(C.Structure):
    _fields_ = [("pages", C.c_void_p), ("npages", C.c_uint32), ("page_sz", C.c_uint32),
                ("flags", C.c_uint32), ("attr_off", C.c_int32), ("attr_width", C.c_int32),
                ("lo", C.c_int64), ("hi", C.c_int64), ("out_items", C.c_void_p),
                ("out_cap", C.c_uint32), ("out_count", C.c_void_p), ("page_status", C.c_void_p),
                ("blkno_base", C.c_uint32), ("blknos", C.c_void_p)]


class PgMvcc(C.Structure):
    """strom_pg_mvcc (strom.h): snapshot, own transaction and SLRU windows."""
    _fields_ = [("xmin", C.c_uint32), ("xmax", C.c_uint32), ("xip", C.c_void_p),
                ("nxip", C.c_uint32), ("suboverflowed", C.c_uint32), ("subxip", C.c_void_p),
                ("nsubxip", C.c_uint32), ("curcid", C.c_uint32), ("curxids", C.c_void_p),
                ("ncurxids", C.c_uint32), ("clog_base", C.c_uint32), ("clog", C.c_void_p),
                ("clog_n", C.c_uint64), ("subtrans", C.c_void_p), ("subtrans_base", C.c_uint32),
                ("subtrans_n", C.c_uint32), ("mx_offsets", C.c_void_p), ("mx_base", C.c_uint32),
                ("mx_n", C.c_uint32), ("mx_members", C.c_void_p), ("mxm_n", C.c_uint64),
                ("mxm_base", C.c_uint32), ("pad", C.c_uint32)]


HEAP_MAX_ATTS = 64
HEAP_MAX_QUALS = 8


class HeapTupDesc(C.Structure):
    _fields_ = [("natts", C.c_int32), ("attlen", C.c_int16 * HEAP_MAX_ATTS),
                ("attalign", C.c_uint8 * HEAP_MAX_ATTS), ("cacheoff", C.c_int16 * HEAP_MAX_ATTS)]


class HeapQual(C.Structure):
    _fields_ = [("attno", C.c_int16), ("kind", C.c_uint8), ("nconst", C.c_uint8),
                ("pad", C.c_uint32), ("lo", C.c_int64), ("hi", C.c_int64),
                ("cbytes", C.c_uint8 * 32)]


class HeapQual2(C.Structure):
    """strom_heap_qual2: one qualifier of a CNF program (constants in a pool)."""
    _fields_ = [("attno", C.c_int16), ("kind", C.c_uint8), ("flags", C.c_uint8),
                ("clause", C.c_uint32), ("nconst", C.c_uint32), ("coff", C.c_uint32),
                ("lo", C.c_int64), ("hi", C.c_int64)]


class HeapScan2Args(C.Structure):
    _fields_ = [("base", HeapScanArgs), ("desc", HeapTupDesc), ("nquals", C.c_int32),
                ("quals", HeapQual * HEAP_MAX_QUALS), ("recheck_count", C.c_void_p),
                ("prog", C.c_void_p), ("cpool", C.c_void_p), ("nprog", C.c_uint32),
                ("cpool_len", C.c_uint32), ("mvcc", PgMvcc), ("mvcc_pages", C.c_void_p),
                ("mvcc_removed", C.c_void_p), ("mvcc_on", C.c_uint32),
                ("mvcc_running_bits", C.c_uint32), ("mvcc_running", C.c_void_p)]


class DecompDesc(C.Structure):
    _fields_ = [("src_off", C.c_uint64), ("dst_off", C.c_uint64), ("src_len", C.c_uint32),
                ("dst_len", C.c_uint32)]


# ----------------------------------------------------------------- loading
_lib = None
_lock = threading.Lock()

_SIGS = {
    "strom_version": (C.c_char_p, []),
    "strom_provider": (C.c_int, []),
    "strom_open": (C.c_int, []),
    "strom_close": (C.c_int, [C.c_int]),
    "strom_ioctl": (C.c_int, [C.c_int, C.c_ulong, C.c_void_p]),
    "nvme_strom_ioctl": (C.c_int, [C.c_ulong, C.c_void_p]),
    "strom_pread_gpu": (C.c_long, [C.c_int, C.c_ulong, C.c_size_t, C.c_int, C.c_uint64,
                                   C.c_uint64]),
    "strom_pread_gpu_lat": (C.c_int, [C.c_int, C.c_ulong, C.c_size_t, C.c_int, C.c_void_p,
                                      C.c_uint32, C.c_uint64, C.c_void_p]),
    "strom_ioctl_lat": (C.c_int, [C.c_int, C.c_ulong, C.c_size_t, C.c_int, C.c_void_p,
                                  C.c_uint32, C.c_uint64, C.c_void_p]),
    "strom_pread_gpu_phases": (C.c_int, [C.c_int, C.c_ulong, C.c_size_t, C.c_int, C.c_void_p,
                                         C.c_uint32, C.c_uint64, C.c_void_p]),
    "strom_pread_raw_lat": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p]),
    "strom_pread_pair_lat": (C.c_int, [C.c_int, C.c_ulong, C.c_size_t, C.c_int, C.c_void_p,
                                       C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p]),
    "strom_raw_read_rate": (C.c_int, [C.c_int, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "strom_raw_read_list": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                      C.c_uint32, C.c_int, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double)]),
    "strom_export_dmabuf": (C.c_int, [C.c_uint64, C.c_uint64, C.POINTER(C.c_int),
                                      C.POINTER(C.c_uint64)]),
    "strom_ingest_info": (C.c_int, [C.c_int, C.c_void_p]),
    "strom_dmabuf_mmap": (C.c_void_p, [C.c_int, C.c_size_t]),
    "strom_dmabuf_munmap": (C.c_int, [C.c_void_p, C.c_size_t]),
    "strom_dmabuf_gc": (C.c_int, []),
    "strom_stripe_open": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64]),
    "strom_stripe_close": (C.c_int, [C.c_int]),
    "strom_register_file": (C.c_int, [C.c_int]),
    "strom_unregister_file": (C.c_int, [C.c_int]),
    "strom_gpu_detached": (C.c_long, []),
    "strom_gpu_bar_bytes": (C.c_long, [C.c_ulong]),
    "strom_host_costs": (C.c_int, [C.c_int, C.c_void_p, C.c_int]),
    "strom_engine_costs": (C.c_int, [C.c_ulong, C.c_int, C.c_void_p, C.c_int]),
    "strom_config_set": (C.c_int, [C.c_char_p, C.c_char_p]),
    "strom_config_get": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t]),
    "strom_engine_reset": (C.c_int, []),
    "strom_fault_inject": (C.c_int, [C.c_long, C.c_int, C.c_long, C.c_int, C.c_int]),
    "strom_fake_backend": (C.c_int, [C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "strom_resident_bytes": (C.c_long, [C.c_int, C.c_uint64, C.c_uint64]),
    "strom_evict_file": (C.c_int, [C.c_int]),
    "strom_crc32c_host": (C.c_uint32, [C.c_uint32, C.c_void_p, C.c_size_t]),
    "strom_raid0_map": (C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_int), C.c_int, C.c_uint32,
                                  C.POINTER(C.c_uint64), C.c_int, C.c_uint64, C.c_uint32,
                                  C.POINTER(C.c_int), C.POINTER(C.c_uint64)]),
    "strom_lz4_compress_host": (C.c_long, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]),
    "strom_lz4_decompress_host": (C.c_long, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]),
    "strom_snappy_compress_host": (C.c_long, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]),
    "strom_snappy_decompress_host": (C.c_long, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]),
    "strom_pg_checksum_host": (C.c_uint16, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "strom_pg_apply_mvcc": (C.c_long, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                       C.c_uint32, C.c_void_p]),
    "strom_pg_tuple_visible": (C.c_int, [C.c_void_p, C.c_void_p]),
    "strom_pg_read_check_pages": (C.c_long, [C.c_int, C.c_void_p, C.c_uint32, C.c_uint32,
                                             C.c_uint32, C.c_void_p, C.c_void_p, C.c_int,
                                             C.c_void_p]),
    "strom_heap_scan_mvcc": (C.c_int, [C.POINTER(HeapScanArgs), C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_void_p]),
    "strom_pg_apply_snapshot": (C.c_long, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]),
    "strom_atomic_fetch_add_u64": (C.c_uint64, [C.c_void_p, C.c_uint64]),
    "strom_atomic_cas_u64": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64]),
    "strom_atomic_load_u64": (C.c_uint64, [C.c_void_p]),
    "strom_gpu_count": (C.c_int, []),
    "strom_crc32c_chunks": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]),
    "strom_crc32c_combine": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64,
                                       C.c_void_p, C.c_void_p]),
    "strom_chunk_scatter": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                      C.c_uint32, C.c_void_p]),
    "strom_chunk_gather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.c_uint32, C.c_void_p]),
    "strom_verify_pattern": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                       C.c_void_p]),
    "strom_verify_equal": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                     C.c_void_p]),
    "strom_fill_pattern": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]),
    "strom_heap_scan": (C.c_int, [C.POINTER(HeapScanArgs), C.c_void_p]),
    "strom_heap_scan2": (C.c_int, [C.POINTER(HeapScan2Args), C.c_void_p]),
    "strom_heap_prog_check": (C.c_int, [C.POINTER(HeapTupDesc), C.c_void_p, C.c_uint32,
                                        C.c_char_p, C.c_uint32]),
    "strom_heap_project": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.POINTER(HeapTupDesc), C.c_int, C.c_int, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    "strom_heap_project_n": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.POINTER(HeapTupDesc), C.c_void_p, C.c_uint32,
                                       C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "strom_decompress": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                   C.c_void_p, C.c_void_p]),
    "strom_column_filter": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_double,
                                      C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]),
    "strom_bitmap_to_indices": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                          C.c_void_p]),
    "strom_column_filter_batched": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_uint64,
                                              C.c_double, C.c_double, C.c_void_p, C.c_void_p,
                                              C.c_void_p]),
    "strom_bitmap_to_rows": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                       C.c_void_p, C.c_void_p, C.c_void_p]),
    "strom_column_filter_batched2": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_uint64,
                                               C.c_double, C.c_double, C.c_void_p, C.c_void_p,
                                               C.c_int, C.c_void_p]),
    "strom_bitmap_to_rows_proj": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                            C.c_void_p, C.c_void_p, C.c_void_p]),
    "strom_column_qual": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p,
                                    C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "strom_bitmap_to_rows_str": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p]),
    "strom_io_info": (C.c_int, [C.c_void_p]),
    "strom_io_prof": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "strom_arrow_headers": (C.c_int, [C.c_int, C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_int32, C.c_void_p]),
    "strom_zstd_host": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
    "strom_zstd_host_fp": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                     C.c_uint32]),
    "strom_zstd_scratch_sizes": (None, [C.c_void_p]),
    "strom_zstd_host_fp_stats": (None, [C.c_void_p]),
    "strom_zstd_fp_mode": (C.c_int, [C.c_int]),
    "strom_zstd_scratch_keep": (C.c_uint32, []),
    "strom_zstd_fp_per_cu": (C.c_uint32, []),
    "strom_decompress_zstd_mode": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64,
                                             C.c_void_p, C.c_int]),
    "strom_decompress_zstd": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "strom_zstd_lds_bytes": (C.c_uint32, []),
    "strom_decompress_zstd_lp": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p]),
    "strom_zstd_lp_info": (None, [C.c_void_p]),
    "strom_zstd_lp_last": (C.c_int, [C.c_void_p, C.c_void_p]),
    "strom_zstd_host_lp": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                     C.c_void_p, C.c_double]),
    "strom_zstd_release": (C.c_int, []),
    "strom_lz4par_host": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                    C.c_void_p]),
    "strom_decompress_par": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_void_p, C.c_void_p]),
    "strom_decompress_par512": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_void_p, C.c_void_p]),
    "strom_decompress_par512b": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.c_void_p, C.c_void_p]),
    "strom_decompress_lanes": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_void_p]),
    "strom_file_topology": (C.c_int, [C.c_int, C.c_void_p]),
    "strom_gpu_pci_bdf": (C.c_int, [C.c_int, C.c_char_p, C.c_size_t]),
}


class NativeMissing(ImportError):
    pass


def lib():
    """Load libstrom.so from the package tree (raises NativeMissing if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeMissing(
                f"{LIB_PATH} not built: run `make -j16` or `python -m nvme_strom_amd.build`")
        handle = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL, use_errno=True)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def has(name: str) -> bool:
    return getattr(lib(), name, None) is not None
