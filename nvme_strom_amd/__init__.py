"""nvme_strom_amd — MI355X-native SSD→HBM direct-storage engine.

Capabilities of nvme-strom (reference: kmod/, utils/, pgsql/) re-designed
for CDNA4 + ROCm:

- ``api``       ioctl-compatible engine surface (CHECK_FILE, MAP/UNMAP/LIST/
                INFO_GPU_MEMORY, ALLOC_DMA_BUFFER, MEMCPY_SSD2GPU/SSD2RAM,
                MEMCPY_WAIT, STAT_INFO) backed by libstrom (C++ engine).
- ``tensor``    HBM buffers as PyTorch-ROCm tensors, file → tensor loaders.
- ``ops``       hand-written HIP kernels: CRC32C verify, chunk reorder,
                PG heap-page scan + checksum, LZ4/snappy decode, column filter.
- ``models``    end-to-end pipelines: streaming SSD→HBM loader (nvme_test),
                SSD→RAM loader (ssd2ram_test), PG heap scan, Arrow IPC scan.
- ``parallel``  one-process-per-GPU shard loading + RCCL fan-out over xGMI.
- ``utils``     stats viewer (nvme_stat), NUMA helpers, test-file helpers.
"""
from .api import (  # noqa: F401
    CopyResult, DmaBuffer, FileInfo, GpuMapping, Session, StromError, alloc_dma_buffer,
    check_file, config_get, config_set, configure, crc32c_host, dmabuf_gc, engine_reset, evict_file,
    gpu_detached,
    fake_backend, fault_inject, hist_percentile, info_gpu_memory, list_gpu_memory, map_gpu_memory,
    memcpy_ssd2gpu, memcpy_ssd2ram, memcpy_wait, pread_gpu, pread_gpu_latency, provider,
    EXTENT_DTYPE, ExtentResult, extents_array, memcpy_ssd2gpu_extents,
    PHASES, host_costs, engine_costs, ingest_info, io_info, io_prof, ioctl_latency, phase_breakdown, pread_gpu_phases, pread_raw_latency, pread_pair_latency, raw_read_rate, raw_read_list,
    resident_bytes, session, StripeSet, RegisteredFile, write_striped,
    stat_hist, stat_info, unmap_gpu_memory, version,
)

__version__ = "0.1.0"
